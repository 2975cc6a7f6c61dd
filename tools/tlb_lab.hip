// TLB lab: does a one-shot weight read (a decode GEMV's access pattern: every byte read once,
// from memory no recent kernel touched) start faster when its pages were translated just
// before?  For each 48 MiB region r of a 6 GiB buffer (regions visited in a scattered
// order, so neither the data nor the translations are warm):
//   touch(r or a control region) -> read(r), the read timed by events.
// `touch` loads one dword per STRIDE bytes of the region, from a workgroup on every XCD
// (blockIdx % 8 round-robin placement), i.e. it warms translations, not data.
//   hipcc --offload-arch=gfx950 -O3 tools/tlb_lab.hip -o tools/tlb_lab.bin
#include <hip/hip_runtime.h>

#include <stdio.h>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      printf("%s failed: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// one-shot read: grid-stride 16-B nt loads, 8 in flight per lane
__global__ __launch_bounds__(512) void read_kernel(const u32x4* __restrict__ p, long n16, unsigned* sink) {
  u32x4 acc = {0, 0, 0, 0};
  const long stride = (long)gridDim.x * blockDim.x;
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 7 * stride < n16; i += 8 * stride) {
    u32x4 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = __builtin_nontemporal_load(p + i + k * stride);
#pragma unroll
    for (int k = 0; k < 8; ++k) acc ^= v[k];
  }
  for (; i < n16; i += stride) acc ^= __builtin_nontemporal_load(p + i);
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9e3779b9u) sink[0] = 1;
}

// translation warm-up: workgroup w (of 8 * per_xcd) touches every (per_xcd)-th page
__global__ void touch_kernel(const unsigned* __restrict__ p, long bytes, long page, int per_xcd, unsigned* sink) {
  const int xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
  (void)xcd;
  unsigned acc = 0;
  for (long off = ((long)j * 64 + threadIdx.x) * page; off < bytes; off += (long)per_xcd * 64 * page)
    acc ^= __builtin_nontemporal_load(p + off / 4);
  if (acc == 0x9e3779b9u) sink[0] = 1;
}

int main() {
  const long REG = 48l << 20, NREG = 128, TOTAL = REG * NREG;  // 6 GiB
  char* buf;
  unsigned* sink;
  CK(hipMalloc(&buf, TOTAL));
  CK(hipMalloc(&sink, 256));
  CK(hipMemset(buf, 1, TOTAL));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  const long pages[] = {4096, 65536, 2l << 20};
  for (int pi = 0; pi < 3; ++pi) {
    for (int mode = 0; mode < 3; ++mode) {  // 0: no touch, 1: touch a control region, 2: touch r
      double tot = 0;
      int cnt = 0;
      for (int it = 0; it < 48; ++it) {
        const long r = (it * 37 + mode * 11 + pi * 5) % NREG;
        const long c = (r + NREG / 2) % NREG;
        const char* reg = buf + r * REG;
        if (mode) {
          const char* t = buf + (mode == 2 ? r : c) * REG;
          hipLaunchKernelGGL(touch_kernel, dim3(8 * 4), dim3(64), 0, s, (const unsigned*)t, REG, pages[pi], 4, sink);
        }
        CK(hipEventRecord(e0, s));
        hipLaunchKernelGGL(read_kernel, dim3(1024), dim3(512), 0, s, (const u32x4*)reg, REG / 16, sink);
        CK(hipEventRecord(e1, s));
        CK(hipStreamSynchronize(s));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (it >= 8) {
          tot += ms;
          ++cnt;
        }
      }
      printf("page %7ld  mode %s: read 48 MiB one-shot %.2f us (%.2f TB/s)\n", pages[pi],
             mode == 0 ? "no touch     " : (mode == 1 ? "touch control" : "touch region "), tot / cnt * 1e3,
             REG / (tot / cnt * 1e-3) / 1e12);
    }
  }
  return 0;
}
