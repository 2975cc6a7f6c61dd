// Peak probes for the roofline ("peaks ... are re-measured by a STREAM-like
// copy and an MFMA loop microbenchmark on the box, and both are reported").  Not on the span
// path: bench.py times them beside the workload and reports them next to the spec peaks.
//   * hbm read : a streaming read of a buffer far larger than the 256 MiB Infinity Cache,
//                16 B per lane, 8 loads in flight per lane (tools/bw_probe.hip's best shape)
//   * mfma     : v_mfma_f32_16x16x32_bf16 chains from registers, 8 independent accumulators per
//                wave, two waves per SIMD -- the dense bf16 rate the prefill kernels use
#include "../../include/inferd_span.h"
#include "common.h"
#include "kernels.h"

// (built with -mllvm -amdgpu-mfma-vgpr-form, Makefile: accumulators stay in VGPRs; the AGPR
// form copies the loop-carried chains through v_accvgpr moves every iteration)

namespace {

typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));

// workgroup w streams its own contiguous run of `tiles_per_wg` 1 KiB tiles (one tile = one
// 16-B-per-lane wave load); its 8 waves take every 8th tile, 8 loads in flight per lane
__global__ __launch_bounds__(512) void probe_read_kernel(const u32x4_t* __restrict__ p, int64_t tiles_per_wg,
                                                         unsigned* __restrict__ sink) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const u32x4_t* base = p + blockIdx.x * tiles_per_wg * 64 + lane;
  u32x4_t acc = {0u, 0u, 0u, 0u};
  int64_t t = wave;
  for (; t + 7 * 8 < tiles_per_wg; t += 8 * 8) {
    u32x4_t v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = base[(t + u * 8) * 64];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc ^= v[u];
  }
  for (; t < tiles_per_wg; t += 8) acc ^= base[t * 64];
  // never true for the probe's fill; keeps the loads live (vector store)
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9e3779b9u) sink[threadIdx.x] = acc.x;
}

__global__ __launch_bounds__(256) void probe_mfma_kernel(int iters, float* __restrict__ sink) {
  bf16x8 a, b;
#pragma unroll
  for (int j = 0; j < 8; ++j) {  // random-looking operands in [-1, 1): the clock the chip holds
    // on random data is lower than on zeros (MI355X_MICROARCH.md, DVFS), as in the GEMMs
    const unsigned h = (threadIdx.x * 0x9e3779b1u + j * 0x85ebca77u + blockIdx.x * 0xc2b2ae3du) ^ 0x27d4eb2fu;
    const unsigned h2 = h * 0x165667b1u + 0x61c88647u;
    a[j] = (__bf16)((float)(h >> 8) * (2.0f / 16777216.0f) - 1.0f);
    b[j] = (__bf16)((float)(h2 >> 8) * (2.0f / 16777216.0f) - 1.0f);
  }
  f32x4 acc[8];
  const float t = (float)threadIdx.x;
#pragma unroll
  for (int c = 0; c < 8; ++c) acc[c] = f32x4{t, t + 1.f, t + 2.f, t + (float)c};
  for (int it = 0; it < iters; it += 4) {  // iters: a multiple of 4 (launcher)
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int c = 0; c < 8; ++c) acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[c], 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < 8; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
  if (s == -1.0f) sink[threadIdx.x] = s;  // never true; keeps the chains live (vector store)
}

}  // namespace

extern "C" int inferd_probe_hbm_read(const void* buf, int64_t bytes, void* sink, int32_t n_wg, void* stream) {
  if (!buf || !sink || bytes < 16 || n_wg < 1) return inferd_fail(INFERD_ERR_ARG, "probe_hbm_read: bad arguments");
  const int64_t per = bytes / 1024 / n_wg;
  if (per < 1) return inferd_fail(INFERD_ERR_ARG, "probe_hbm_read: fewer than one KiB per workgroup");
  hipLaunchKernelGGL(probe_read_kernel, dim3(n_wg), dim3(512), 0, (hipStream_t)stream, (const u32x4_t*)buf, per,
                     (unsigned*)sink);
  return hipGetLastError() == hipSuccess ? INFERD_OK : inferd_fail(INFERD_ERR_HIP, "probe_hbm_read: launch failed");
}

extern "C" int inferd_probe_mfma(int32_t iters, int32_t n_wg, void* sink, void* stream, double* flops) {
  if (!sink || iters < 4 || iters % 4 || n_wg < 1)
    return inferd_fail(INFERD_ERR_ARG, "probe_mfma: bad arguments (iters: a positive multiple of 4)");
  hipLaunchKernelGGL(probe_mfma_kernel, dim3(n_wg), dim3(256), 0, (hipStream_t)stream, iters, (float*)sink);
  if (flops) *flops = (double)n_wg * 4 /* waves */ * iters * 8 /* chains */ * (2.0 * 16 * 16 * 32);
  return hipGetLastError() == hipSuccess ? INFERD_OK : inferd_fail(INFERD_ERR_HIP, "probe_mfma: launch failed");
}
