// Persistent-MLP feasibility lab (standalone; not part of the engine).  Prices the decode
// layer's gate/up -> down seam as byte streams only, so the numbers bound what a persistent
// MLP kernel could save before any GEMM is written:
//   two  : phase A (201 MB, the gate/up weights) and phase B (100.7 MB, down) as two launches,
//          256 workgroups x 8 waves, each workgroup a contiguous run (the GEMV read shape)
//   one  : ONE launch, 256 workgroups (one per CU: 128 KiB of LDS each), phase A, then an
//          arrival on a device counter and a bounded wait for all 256, then phase B
//   pre  : as `one`, but before waiting each workgroup LDS-DMAs the first 128 KiB of its
//          phase-B run (bytes that do not depend on phase A) and reads them back after
//   sharded: `pre` with the counter split per XCD (8 counters; XCD leader adds to the top)
// Rotates 4 weight sets (1.2 GB) so no launch reuses the Infinity Cache.
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 tools/mk_lab.hip -o /tmp/mk_lab && /tmp/mk_lab
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x)                                                                \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
constexpr int NW = 8;
constexpr int PRE_KB = 128;

// one workgroup reads `tiles` contiguous KiB tiles at p (8 waves, every 8th tile, 8 in flight)
__device__ __forceinline__ u32x4 read_run(const u32x4* __restrict__ p, int64_t tiles, int64_t t0) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const u32x4* base = p + lane;
  u32x4 acc = {0u, 0u, 0u, 0u};
  int64_t t = t0 + wave;
  for (; t + 7 * NW < tiles; t += 8 * NW) {
    u32x4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = __builtin_nontemporal_load(base + (t + u * NW) * 64);
#pragma unroll
    for (int u = 0; u < 8; ++u) acc ^= v[u];
  }
  for (; t < tiles; t += NW) acc ^= __builtin_nontemporal_load(base + t * 64);
  return acc;
}

__global__ __launch_bounds__(512) void read_kernel(const u32x4* __restrict__ p, int64_t tiles_per_wg,
                                                   unsigned* __restrict__ sink) {
  const u32x4 acc = read_run(p + blockIdx.x * tiles_per_wg * 64, tiles_per_wg, 0);
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9e3779b9u) sink[threadIdx.x] = acc.x;
}

// The GEMV's read shape: wave w takes batches w, w + 8, ... of TW consecutive KiB tiles, DEPTH
// batches in flight; WITH_A also reads the batch's activation fragments (TW KiB of a buffer
// every workgroup shares, L2-resident: the 16 x K bf16 rows a decode GEMV streams beside W)
// ROWMAJOR: the activations as the engine stores them, 16 rows of K bf16 (lane l reads row
// l % 16, 16 B at k-offset 8 (l / 16) of each 32-wide k-tile); otherwise fragment-packed
// (each k-tile's 1 KiB contiguous, as the weights)
template <bool WITH_A, int TW, int DEPTH, bool ROWMAJOR = false, int NWT = NW>
__global__ __launch_bounds__(NWT * 64) void read_wa_kernel(const u32x4* __restrict__ p, const u32x4* __restrict__ act,
                                                      int64_t tiles_per_wg, unsigned* __restrict__ sink) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const u32x4* base = p + blockIdx.x * tiles_per_wg * 64 + lane;
  // row-major: element offset row * K + 8 * (lane / 16), in 16-B units row * K / 8 + lane / 16;
  // a k-tile advances 32 elements = 4 units (the "* 64" below is then scaled back by 16)
  const u32x4* abase = ROWMAJOR ? act + (int64_t)(lane & 15) * (tiles_per_wg * 4) + (lane >> 4) : act + lane;
  constexpr int ASTEP = ROWMAJOR ? 4 : 64;
  u32x4 acc = {0u, 0u, 0u, 0u};
  const int64_t nb = tiles_per_wg / TW;
  for (int64_t b0 = wave; b0 < nb; b0 += (int64_t)NWT * DEPTH) {
    u32x4 v[DEPTH][TW], a[DEPTH][TW];
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      const int64_t b = b0 + d * NWT;
      if (b < nb) {
#pragma unroll
        for (int u = 0; u < TW; ++u) {
          if constexpr (WITH_A) a[d][u] = abase[(b * TW + u) * ASTEP];
          v[d][u] = __builtin_nontemporal_load(base + (b * TW + u) * 64);
        }
      } else {
#pragma unroll
        for (int u = 0; u < TW; ++u) v[d][u] = a[d][u] = u32x4{0u, 0u, 0u, 0u};
      }
    }
#pragma unroll
    for (int d = 0; d < DEPTH; ++d)
#pragma unroll
      for (int u = 0; u < TW; ++u) {
        acc ^= v[d][u];
        if constexpr (WITH_A) acc += a[d][u];
      }
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9e3779b9u) sink[threadIdx.x] = acc.x;
}

// MODE 0: no prefetch; 1: LDS-DMA prefetch of phase B's first PRE_KB KiB; SHARD: per-XCD counters
template <int MODE, bool SHARD>
__global__ __launch_bounds__(512, 1) void persist_kernel(const u32x4* __restrict__ pa, int64_t ta,
                                                         const u32x4* __restrict__ pb, int64_t tb,
                                                         unsigned* __restrict__ ctr, unsigned target,
                                                         unsigned* __restrict__ sink) {
  __shared__ __attribute__((aligned(16))) char lds[PRE_KB * 1024];
  __shared__ int ok;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  u32x4 acc = read_run(pa + blockIdx.x * ta * 64, ta, 0);
  const u32x4* myb = pb + blockIdx.x * tb * 64;
  if constexpr (MODE == 1) {
    // PRE_KB tiles of phase B into LDS: wave w takes tiles w, w + 8, ...
    for (int t = wave; t < PRE_KB; t += NW)
      __builtin_amdgcn_global_load_lds((const void*)(myb + t * 64 + lane), (void*)(lds + t * 1024), 16, 0, 0);
  }
  // arrival: phase A's results would be stored write-through here; then one add per workgroup
  __syncthreads();
  if (threadIdx.x == 0) {
    if constexpr (SHARD) {
      const unsigned x = blockIdx.x & 7;  // round-robin XCD of this workgroup
      const unsigned prev = __hip_atomic_fetch_add(&ctr[16 * (1 + x)], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((prev + 1) % (gridDim.x / 8) == 0)  // last of its XCD: one add to the top counter
        __hip_atomic_fetch_add(&ctr[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      int budget = 1 << 20;
      while (__hip_atomic_load(&ctr[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target / (gridDim.x / 8) &&
             --budget > 0)
        __builtin_amdgcn_s_sleep(1);
      ok = budget > 0;
    } else {
      __hip_atomic_fetch_add(&ctr[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      int budget = 1 << 20;
      while (__hip_atomic_load(&ctr[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target && --budget > 0)
        __builtin_amdgcn_s_sleep(1);
      ok = budget > 0;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
  if (!ok) {
    if (threadIdx.x == 0) sink[1023] = 1u;  // timed out: flag, never hang
    return;
  }
  if constexpr (MODE == 1) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int t = wave; t < PRE_KB; t += NW) acc ^= *(const u32x4*)(lds + t * 1024 + lane * 16);
    acc ^= read_run(myb, tb, PRE_KB);
  } else {
    acc ^= read_run(myb, tb, 0);
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9e3779b9u) sink[threadIdx.x] = acc.x;
}

int main() {
  int dev = 0, cus = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const int G = 256;
  if (cus < G) {
    printf("needs %d CUs, device has %d: skipped\n", G, cus);
    return 0;
  }
  // per workgroup: phase A 768 KiB (201.3 MB / 256), phase B 384 KiB (100.7 MB / 256)
  const int64_t ta = 768, tb = 384;
  const int ROT = 4;
  const size_t bytes_a = (size_t)G * ta * 1024, bytes_b = (size_t)G * tb * 1024;
  u32x4 *A[ROT], *B[ROT];
  for (int r = 0; r < ROT; ++r) {
    CHECK(hipMalloc((void**)&A[r], bytes_a));
    CHECK(hipMalloc((void**)&B[r], bytes_b));
    CHECK(hipMemset(A[r], 1 + r, bytes_a));
    CHECK(hipMemset(B[r], 2 + r, bytes_b));
  }
  unsigned *sink, *ctr;
  CHECK(hipMalloc((void**)&sink, 4096));
  CHECK(hipMalloc((void**)&ctr, 4096));
  CHECK(hipMemset(sink, 0, 4096));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int N = 40;
  auto time = [&](const char* name, auto launch) {
    CHECK(hipMemset(ctr, 0, 4096));
    unsigned gen = 0;
    for (int i = 0; i < 8; ++i) launch(i % ROT, ++gen);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    for (int i = 0; i < N; ++i) launch(i % ROT, ++gen);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    unsigned flag = 0;
    CHECK(hipMemcpy(&flag, sink + 1023, 4, hipMemcpyDeviceToHost));
    const double us = ms * 1e3 / N;
    printf("  %-34s %8.2f us  %7.0f GB/s%s\n", name, us, (bytes_a + bytes_b) / (us * 1e-6) / 1e9,
           flag ? "  (WAIT TIMED OUT)" : "");
    return flag;
  };
  printf("phase A %.1f MB + phase B %.1f MB, %d workgroups\n", bytes_a / 1e6, bytes_b / 1e6, G);
  u32x4* act;
  CHECK(hipMalloc((void**)&act, (size_t)ta * 1024));
  CHECK(hipMemset(act, 3, (size_t)ta * 1024));
  // W-only floors in each decode GEMV's own grid shape (packed A beside W where it reads one)
  for (int rep = 0; rep < 2; ++rep) {
    time("o shape: 256 WG x 8w, 128 KiB, W", [&](int r, unsigned) {
      hipLaunchKernelGGL((read_wa_kernel<false, 4, 3>), dim3(256), dim3(512), 0, 0, B[r], act, 128, sink);
    });
    time("o shape: + packed A", [&](int r, unsigned) {
      hipLaunchKernelGGL((read_wa_kernel<true, 4, 3>), dim3(256), dim3(512), 0, 0, B[r], act, 128, sink);
    });
    time("qkv shape: 768 WG x 4w, 64 KiB, W", [&](int r, unsigned) {
      hipLaunchKernelGGL((read_wa_kernel<false, 4, 3, false, 4>), dim3(768), dim3(256), 0, 0, A[r], act, 64, sink);
    });
    time("qkv shape: + packed A", [&](int r, unsigned) {
      hipLaunchKernelGGL((read_wa_kernel<true, 4, 3, false, 4>), dim3(768), dim3(256), 0, 0, A[r], act, 64, sink);
    });
    time("gate/up shape: 768 WG x 4w, 256 KiB, W", [&](int r, unsigned) {
      hipLaunchKernelGGL((read_wa_kernel<false, 8, 2, false, 4>), dim3(768), dim3(256), 0, 0, A[r], act, 256, sink);
    });
  }
  for (int rep = 0; rep < 2; ++rep) {
    time("B as GEMV reads W   (TW4 D3)", [&](int r, unsigned) {
      hipLaunchKernelGGL((read_wa_kernel<false, 4, 3>), dim3(G), dim3(512), 0, 0, B[r], act, tb, sink);
    });
    time("B as GEMV reads W+A (TW4 D3)", [&](int r, unsigned) {
      hipLaunchKernelGGL((read_wa_kernel<true, 4, 3>), dim3(G), dim3(512), 0, 0, B[r], act, tb, sink);
    });
    time("B as GEMV reads W+A row-major (TW4 D3)", [&](int r, unsigned) {
      hipLaunchKernelGGL((read_wa_kernel<true, 4, 3, true>), dim3(G), dim3(512), 0, 0, B[r], act, tb, sink);
    });
    time("B as GEMV reads W+A (TW4 D2)", [&](int r, unsigned) {
      hipLaunchKernelGGL((read_wa_kernel<true, 4, 2>), dim3(G), dim3(512), 0, 0, B[r], act, tb, sink);
    });
    time("B as GEMV reads W+A (TW2 D4)", [&](int r, unsigned) {
      hipLaunchKernelGGL((read_wa_kernel<true, 2, 4>), dim3(G), dim3(512), 0, 0, B[r], act, tb, sink);
    });
    time("B as GEMV reads W+A (TW8 D2)", [&](int r, unsigned) {
      hipLaunchKernelGGL((read_wa_kernel<true, 8, 2>), dim3(G), dim3(512), 0, 0, B[r], act, tb, sink);
    });
  }
  for (int rep = 0; rep < 2; ++rep) {
    time("A alone", [&](int r, unsigned) {
      hipLaunchKernelGGL(read_kernel, dim3(G), dim3(512), 0, 0, A[r], ta, sink);
    });
    time("B alone", [&](int r, unsigned) {
      hipLaunchKernelGGL(read_kernel, dim3(G), dim3(512), 0, 0, B[r], tb, sink);
    });
    time("two launches (A then B)", [&](int r, unsigned) {
      hipLaunchKernelGGL(read_kernel, dim3(G), dim3(512), 0, 0, A[r], ta, sink);
      hipLaunchKernelGGL(read_kernel, dim3(G), dim3(512), 0, 0, B[r], tb, sink);
    });
    if (time("one launch, counter wait", [&](int r, unsigned gen) {
          hipLaunchKernelGGL((persist_kernel<0, false>), dim3(G), dim3(512), 0, 0, A[r], ta, B[r], tb, ctr,
                             gen * G, sink);
        }))
      return 1;
    if (time("one launch, B prefetch to LDS", [&](int r, unsigned gen) {
          hipLaunchKernelGGL((persist_kernel<1, false>), dim3(G), dim3(512), 0, 0, A[r], ta, B[r], tb, ctr,
                             gen * G, sink);
        }))
      return 1;
    if (time("one launch, prefetch, XCD counters", [&](int r, unsigned gen) {
          hipLaunchKernelGGL((persist_kernel<1, true>), dim3(G), dim3(512), 0, 0, A[r], ta, B[r], tb, ctr,
                             gen * G, sink);
        }))
      return 1;
  }
  return 0;
}
