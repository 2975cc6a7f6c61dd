// Decode seam lab: the down -> next layer's q/k/v seam of a Qwen3-8B decode
// layer (B = 16) as two launches against ONE persistent launch whose hand-off is
// MI355X_MICROARCH.md's data-tagged granule all-gather (8-byte {tag, value} granules written by
// one sc1 store each, gathered by a flat sc1 sweep on every consumer CU; no counter barrier).
// Read-only weight streams with the engine's byte counts (down 101.3 MB, q/k/v 50.7 MB), no MFMA:
//   * launches : down-like kernel (256 WGs x 8 waves, register ring of 16-B nt loads) writes its
//                16 x 16 output tile (bf16, row-major x[16][4096]); q/k/v-like kernel (768 WGs x 4
//                waves) streams its weights and reads the whole 128 KiB x as 1 KiB A fragments from
//                L2 (one per weight tile, the GEMV's A operand);
//   * granules : one launch, 256 WGs (one per CU) x 8 waves: phase 1 streams the down slice and
//                publishes the tile as 128 granules {epoch, 2 x bf16}; phase 2 issues its q/k/v
//                weight ring prologue (prefetch credit), gathers all 32768 granules (256 KiB) into
//                LDS with sc1 loads, re-reading until every tag is the epoch (bounded: a sweep that
//                gives up sets a flag and the run is reported invalid), then streams its q/k/v
//                slice reading A from LDS;
//   * gather alone: phase 2's all-gather with nothing else running (its cost floor).
// Buffers rotate over 3 sets so no launch finds its weights in the 256 MB Infinity Cache.
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 tools/seam_lab.hip -o tools/labbin/seam_lab
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned long long u64;

constexpr int ROWS = 16, HID = 4096;
constexpr int XBYTES = ROWS * HID * 2;          // 128 KiB of bf16 x
constexpr int NGRAN = ROWS * HID / 2;           // 32768 granules of 2 bf16
constexpr long long DOWN_BYTES = 101318656ll;   // down weights + tails (engine: 101.3 MB)
constexpr long long QKV_BYTES = 50659328ll;     // q/k/v weights (engine: 50.7 MB)

// NW waves stream `bytes` of one workgroup's slice in 1 KiB tiles (wave w: tiles w, w + NW, ...),
// D tiles in flight per wave.  With A (in LDS, or global when a_glob): one 1 KiB A fragment read
// per weight tile, cycling over the 128 KiB of x.  PRE: the first D tiles were issued already.
template <int NW, int D>
__device__ __forceinline__ unsigned stream(const u32x4* base, long long bytes, int wave, int lane, u32x4 (&r)[D],
                                           bool pre, const char* a_lds, const u32x4* a_glob) {
  const long long ntiles = bytes / 1024;
  const long long nper = (ntiles - wave + NW - 1) / NW;
  auto addr = [&](long long j) { return base + (wave + (j < nper ? j : nper - 1) * NW) * 64 + lane; };
  unsigned x = 0;
  if (!pre) {
#pragma unroll
    for (int d = 0; d < D; ++d) r[d] = __builtin_nontemporal_load(addr(d));
  }
  for (long long j = 0; j < nper; j += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int at = (int)((wave + (j + d) * NW) & 127);  // which 1 KiB of x this tile pairs with
      u32x4 a;
      if (a_lds)
        a = *(const u32x4*)(a_lds + at * 1024 + lane * 16);
      else if (a_glob)
        a = a_glob[at * 64 + lane];
      else
        a = u32x4{0, 0, 0, 0};
      x ^= r[d][0] ^ r[d][1] ^ r[d][2] ^ r[d][3] ^ a[0] ^ a[3];
      r[d] = __builtin_nontemporal_load(addr(j + d + D));
    }
  }
  return x;
}

// ---- launches ----------------------------------------------------------------------------------
__global__ __launch_bounds__(512) void down_kernel(const u32x4* w, long long slice, unsigned short* xout,
                                                   unsigned* sink) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  u32x4 r[3];
  const unsigned v = stream<8, 3>(w + (long long)blockIdx.x * slice / 16, slice, wave, lane, r, false, nullptr, nullptr);
  // this workgroup's output tile: columns 16 * blockIdx.x .. +15 of the 16 rows
  if (threadIdx.x < ROWS * 16) {
    const int row = threadIdx.x >> 4, col = blockIdx.x * 16 + (threadIdx.x & 15);
    xout[row * HID + col] = (unsigned short)(v ^ threadIdx.x);
  }
}

__global__ __launch_bounds__(256) void qkv_kernel(const u32x4* w, long long slice, const u32x4* x, unsigned* sink) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  u32x4 r[3];
  const unsigned v = stream<4, 3>(w + (long long)blockIdx.x * slice / 16, slice, wave, lane, r, false, nullptr, x);
  if (v == 0x9e3779b9u) sink[0] = v;
}

// ---- one launch, granule seam -------------------------------------------------------------------
__device__ __forceinline__ void store_granule(u64* g, unsigned epoch, unsigned value) {
  __hip_atomic_store(g, ((u64)value << 32) | epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// MODE 0: phase 1 + gather + q/k/v stream; 1: gather + stream (granules already published);
// 2: stream only (A in LDS, no gather)
template <int MODE>
__global__ __launch_bounds__(512, 1) void seam_kernel(const u32x4* wd, long long sd, const u32x4* wq, long long sq,
                                                      u64* gran, unsigned epoch, unsigned* sink, unsigned* flag) {
  extern __shared__ __attribute__((aligned(16))) char xl[];  // 128 KiB: x gathered
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  u32x4 r[3];
  unsigned v = 0;
  if (MODE == 0) {
    v = stream<8, 3>(wd + (long long)blockIdx.x * sd / 16, sd, wave, lane, r, false, nullptr, nullptr);
    // publish this workgroup's 16 x 16 tile as 128 granules (2 bf16 each): one sc1 8-B store each
    if (threadIdx.x < 128) {
      const int row = threadIdx.x >> 3, cp = threadIdx.x & 7;  // column pair within the tile
      const int gi = (row * HID + blockIdx.x * 16 + 2 * cp) >> 1;
      store_granule(gran + gi, epoch, v ^ threadIdx.x);
    }
  }
  // phase 2: the q/k/v weight ring prologue first (prefetch credit), then the gather
  const u32x4* wb = wq + (long long)blockIdx.x * sq / 16;
  {
    const long long ntiles = sq / 1024;
    const long long nper = (ntiles - wave + 7) / 8;
#pragma unroll
    for (int d = 0; d < 3; ++d) r[d] = __builtin_nontemporal_load(wb + (wave + (d < nper ? d : nper - 1) * 8) * 64 + lane);
  }
  if (MODE < 2) {
    // flat sweep: 512 lanes x 64 granules (granule k * 512 + thread); re-read the stale ones
    u64 pending = ~0ull;
    int spins = 0;
    while (__builtin_amdgcn_ballot_w64(pending != 0) && spins < 100000) {
      if (spins++) __builtin_amdgcn_s_sleep(1);
#pragma unroll 8
      for (int k = 0; k < 64; ++k) {
        if (!(pending >> k & 1)) continue;
        const int gi = k * 512 + threadIdx.x;
        const u64 g = __hip_atomic_load(gran + gi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((unsigned)g == epoch) {
          *(unsigned*)(xl + gi * 4) = (unsigned)(g >> 32);
          pending &= ~(1ull << k);
        }
      }
    }
    if (pending) atomicOr(flag, 1u);
    __syncthreads();
  }
  v ^= stream<8, 3>(wb, sq, wave, lane, r, true, xl, nullptr);
  if (v == 0x9e3779b9u) sink[0] = v;
}

int main() {
  const int ROT = 3;
  std::vector<u32x4*> wd, wq;
  for (int s = 0; s < ROT; ++s) {
    u32x4 *a, *b;
    CHECK(hipMalloc(&a, DOWN_BYTES + (1 << 20)));
    CHECK(hipMalloc(&b, QKV_BYTES + (1 << 20)));
    CHECK(hipMemset(a, 0x11 * (s + 1), DOWN_BYTES + (1 << 20)));
    CHECK(hipMemset(b, 0x21 * (s + 1), QKV_BYTES + (1 << 20)));
    wd.push_back(a);
    wq.push_back(b);
  }
  unsigned short* x;
  u64* gran;
  unsigned *sink, *flag;
  CHECK(hipMalloc(&x, XBYTES));
  CHECK(hipMalloc(&gran, NGRAN * 8));
  CHECK(hipMalloc(&sink, 64));
  CHECK(hipMalloc(&flag, 4));
  CHECK(hipMemset(x, 0, XBYTES));
  CHECK(hipMemset(gran, 0, NGRAN * 8));
  CHECK(hipMemset(flag, 0, 4));
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int ncu = prop.multiProcessorCount;
  printf("CUs %d\n", ncu);
  CHECK(hipFuncSetAttribute((const void*)seam_kernel<0>, hipFuncAttributeMaxDynamicSharedMemorySize, XBYTES));
  CHECK(hipFuncSetAttribute((const void*)seam_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize, XBYTES));
  CHECK(hipFuncSetAttribute((const void*)seam_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize, XBYTES));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  unsigned epoch = 0;
  auto timeit = [&](const char* name, auto fn) {
    for (int i = 0; i < 2 * ROT; ++i) fn(i);
    CHECK(hipDeviceSynchronize());
    const int n = 30 * ROT;
    CHECK(hipEventRecord(e0));
    for (int i = 0; i < n; ++i) fn(2 * ROT + i);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    unsigned f = 0;
    CHECK(hipMemcpy(&f, flag, 4, hipMemcpyDeviceToHost));
    printf("  %-52s %8.2f us%s\n", name, ms * 1e3f / n, f ? "  (A SWEEP GAVE UP: invalid)" : "");
    CHECK(hipMemset(flag, 0, 4));
  };
  const long long sd = DOWN_BYTES / 256 / 1024 * 1024, sq = QKV_BYTES / 768 / 1024 * 1024;
  const long long sq1 = QKV_BYTES / ncu / 8192 * 8192, sd1 = DOWN_BYTES / ncu / 8192 * 8192;
  timeit("down alone (256 x 8 waves)", [&](int i) {
    hipLaunchKernelGGL(down_kernel, dim3(256), dim3(512), 0, 0, wd[i % ROT], sd, x, sink);
  });
  timeit("q/k/v alone (768 x 4 waves, A from L2)", [&](int i) {
    hipLaunchKernelGGL(qkv_kernel, dim3(768), dim3(256), 0, 0, wq[i % ROT], sq, (const u32x4*)x, sink);
  });
  timeit("down alone, ncu x 8 waves (the persistent geometry)", [&](int i) {
    hipLaunchKernelGGL(down_kernel, dim3(ncu), dim3(512), 0, 0, wd[i % ROT], sd1, x, sink);
  });
  timeit("two launches: down -> q/k/v", [&](int i) {
    hipLaunchKernelGGL(down_kernel, dim3(256), dim3(512), 0, 0, wd[i % ROT], sd, x, sink);
    hipLaunchKernelGGL(qkv_kernel, dim3(768), dim3(256), 0, 0, wq[i % ROT], sq, (const u32x4*)x, sink);
  });
  timeit("one launch, granule all-gather seam (ncu x 8 waves)", [&](int i) {
    ++epoch;
    hipLaunchKernelGGL(seam_kernel<0>, dim3(ncu), dim3(512), XBYTES, 0, wd[i % ROT], sd1, wq[i % ROT], sq1, gran,
                       epoch, sink, flag);
  });
  // the all-gather with nothing ahead of it: the granules of the last epoch are all published
  timeit("gather + q/k/v stream only (granules ready)", [&](int i) {
    hipLaunchKernelGGL(seam_kernel<1>, dim3(ncu), dim3(512), XBYTES, 0, wd[i % ROT], sd1, wq[i % ROT], sq1, gran,
                       epoch, sink, flag);
  });
  timeit("q/k/v stream only, ncu x 8 waves, A in LDS (gather skipped)", [&](int i) {
    hipLaunchKernelGGL(seam_kernel<2>, dim3(ncu), dim3(512), XBYTES, 0, wd[i % ROT], sd1, wq[i % ROT], sq1, gran,
                       epoch, sink, flag);
  });
  return 0;
}
