// Lab: v_mfma_f32_32x32x16_bf16 issue rate by operand register file (A/B in VGPR or AGPR,
// accumulator in VGPR or AGPR) and by the distance between dependent MFMAs (independent chains).
// One wave per SIMD, 256 WGs x 4 waves, 4096 MFMAs per wave.  Build: hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

template <int MODE, int CH>
__global__ __launch_bounds__(256, 1) void k(float* out, const bf16x8* in, int iters) {
  bf16x8 a = in[threadIdx.x], b = in[threadIdx.x + 256];
  f32x16 c[CH];
  for (int i = 0; i < CH; ++i) c[i] = f32x16{};
  if constexpr (MODE & 1) asm volatile("" : "+a"(a), "+a"(b));
  if constexpr (MODE & 2)
    for (int i = 0; i < CH; ++i) asm volatile("" : "+a"(c[i]));
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      if constexpr (MODE == 0) asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(c[i]) : "v"(a), "v"(b));
      if constexpr (MODE == 1) asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(c[i]) : "a"(a), "a"(b));
      if constexpr (MODE == 2) asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(c[i]) : "v"(a), "v"(b));
      if constexpr (MODE == 3) asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(c[i]) : "a"(a), "a"(b));
    }
  }
  asm volatile("s_nop 7\n s_nop 7\n s_nop 7");
  float s = 0;
  for (int i = 0; i < CH; ++i) s += c[i][0] + c[i][15];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int MODE, int CH>
void run(float* out, bf16x8* in) {
  const int iters = 4096 / CH;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int w = 0; w < 3; ++w) k<MODE, CH><<<256, 256>>>(out, in, iters);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) k<MODE, CH><<<256, 256>>>(out, in, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double flops = 5.0 * 256 * 4 * 4096 * 32768.0;
  printf("mode %d (A/B %s, C %s) chains %d: %.1f TF/s\n", MODE, MODE & 1 ? "AGPR" : "VGPR", MODE & 2 ? "AGPR" : "VGPR",
         CH, flops / (ms * 1e-3) / 1e12);
}

int main() {
  float* out;
  bf16x8* in;
  hipMalloc(&out, 256 * 256 * 4);
  hipMalloc(&in, 512 * 16);
  unsigned short h[512 * 8];
  for (int i = 0; i < 512 * 8; ++i) h[i] = 0x3c00 + (i * 37 % 200);  // small random-ish bf16
  hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
  run<0, 1>(out, in); run<0, 2>(out, in); run<0, 4>(out, in); run<0, 8>(out, in);
  run<1, 4>(out, in); run<2, 4>(out, in); run<3, 4>(out, in); run<2, 8>(out, in); run<3, 8>(out, in);
  return 0;
}
