// HBM read-bandwidth probe (standalone; not part of the engine).  Streams N bytes with
// 16-B-per-lane loads in the same "one tile = 1 KiB per wave-instruction" shape the skinny
// GEMM uses, for several grid shapes, and reports GB/s.  Build: hipcc --offload-arch=gfx950
// -O3 tools/bw_probe.hip -o /tmp/bw_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// each workgroup streams `per_wg` contiguous KiB tiles; each wave takes every NW-th tile
template <int U>
__global__ void stream_kernel(const u32x4* __restrict__ p, long tiles_per_wg, unsigned* out) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, nw = blockDim.x >> 6;
  const u32x4* base = p + (long)blockIdx.x * tiles_per_wg * 64 + lane;
  u32x4 acc = {0, 0, 0, 0};
  long t = wave;
  for (; t + (long)(U - 1) * nw < tiles_per_wg; t += (long)U * nw) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = base[(t + (long)u * nw) * 64];
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u];
  }
  for (; t < tiles_per_wg; t += nw) acc ^= base[t * 64];
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[0] = 1;
}

int main() {
  const size_t max_bytes = 1ull << 30;
  void* buf;
  unsigned* out;
  hipMalloc(&buf, max_bytes);
  hipMalloc(&out, 4);
  hipMemset(buf, 1, max_bytes);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const double sizes_mb[] = {34.0, 50.6, 100.7, 201.3, 1024.0};
  const int wgs[] = {256, 384, 512, 768, 1024, 2048};
  const int nws[] = {4, 8};
  for (double mb : sizes_mb) {
    for (int nw : nws) {
      for (int g : wgs) {
        long tiles = (long)(mb * 1e6 / 1024);
        long per = tiles / g;
        if (per < 1) continue;
        for (int it = 0; it < 3; ++it)
          hipLaunchKernelGGL(stream_kernel<8>, dim3(g), dim3(nw * 64), 0, 0, (const u32x4*)buf, per, out);
        hipEventRecord(a);
        const int iters = 20;
        for (int it = 0; it < iters; ++it)
          hipLaunchKernelGGL(stream_kernel<8>, dim3(g), dim3(nw * 64), 0, 0, (const u32x4*)buf, per, out);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        double us = ms * 1e3 / iters;
        double gbs = (double)per * g * 1024 / (us * 1e-6) / 1e9;
        printf("%7.1f MB  wg=%5d waves/wg=%d  %8.2f us  %7.1f GB/s\n", per * g * 1024 / 1e6, g, nw, us, gbs);
      }
    }
  }
  return 0;
}
