// Weight-stream lab (read-only): how fast can a decode GEMV's once-read weight bytes be streamed
// on this chip, (A) through a per-wave register ring (the shipped decode GEMVs: 16-B nt loads,
// D batches of TW 1 KiB tiles in flight per wave) versus (B) by LDS-DMA (buffer_load ... lds, nt)
// into a per-wave LDS ring of R batches, consumed by ds_read_b128?  Each workgroup owns one
// contiguous slice (a GEMV's 16-column tile over all of K); wave w takes batches w, w + NW, ...
// Consumption is an XOR (no MFMA): the bytes' landing rate, not the GEMV, is measured.
// Launches rotate over buffers 512 MiB apart (cold: no Infinity Cache hits), HIP events, median.
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 tools/stream_lab.hip -o tools/labbin/stream_lab
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#define CHECK(x)                                                                \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
constexpr int TW = 4;  // 1 KiB tiles per batch

// (A) register ring: D batches in flight per wave
template <int NW, int D>
__global__ __launch_bounds__(NW * 64) void reg_stream(const u32x4* __restrict__ w, long long slice_tiles,
                                                       unsigned* __restrict__ sink) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const u32x4* base = w + (long long)blockIdx.x * slice_tiles * 64 + lane;
  const long long nb = slice_tiles / TW;
  const long long nbw = wave < nb ? (nb - wave + NW - 1) / NW : 0;
  u32x4 r[D][TW];
  unsigned x = 0;
  auto issue = [&](int d, long long j) {
    const long long bb = wave + (j < nbw ? j : nbw - 1) * NW;  // past the end: re-read the last batch
#pragma unroll
    for (int u = 0; u < TW; ++u) r[d][u] = __builtin_nontemporal_load(base + (bb * TW + u) * 64);
  };
  if (nbw == 0) return;
#pragma unroll
  for (int d = 0; d < D - 1; ++d) issue(d, d);
  for (long long j = 0; j < nbw; j += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      issue((d + D - 1) % D, j + d + D - 1);
#pragma unroll
      for (int u = 0; u < TW; ++u) x ^= r[d][u][0] ^ r[d][u][1] ^ r[d][u][2] ^ r[d][u][3];
    }
  }
  sink[blockIdx.x * NW * 64 + threadIdx.x] = x;
}

// (B) LDS-DMA ring: R batches per wave in LDS (4 KiB each), R - 1 in flight while one is read
template <int NW, int R>
__global__ __launch_bounds__(NW * 64) void lds_stream(const u32x4* __restrict__ w, long long slice_tiles,
                                                       unsigned* __restrict__ sink) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  typedef __attribute__((address_space(3))) void* lds_ptr;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int swave = __builtin_amdgcn_readfirstlane(wave);
  const long long nb = slice_tiles / TW;
  const long long nbw = swave < nb ? (nb - swave + NW - 1) / NW : 0;
  if (nbw == 0) return;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(w + (long long)blockIdx.x * slice_tiles * 64), 0, 0x7fffffff, 0x00020000);
  char* ring = lds + swave * R * TW * 1024;
  unsigned x = 0;
  auto issue = [&](int slot, long long j) {
    const long long bb = swave + (j < nbw ? j : nbw - 1) * NW;
#pragma unroll
    for (int u = 0; u < TW; ++u)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr)(ring + (slot * TW + u) * 1024), 16, lane * 16,
                                               (int)((bb * TW + u) * 1024), 0, 2);
  };
#pragma unroll
  for (int d = 0; d < R - 1; ++d) issue(d, d);
  for (long long j = 0; j < nbw; j += R) {
#pragma unroll
    for (int d = 0; d < R; ++d) {
      issue((d + R - 1) % R, j + d + R - 1);
      // batch d landed once all but the (R - 1) * TW youngest loads retired
      if constexpr (R == 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else if constexpr (R == 3) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else if constexpr (R == 4) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
      else if constexpr (R == 6) asm volatile("s_waitcnt vmcnt(20)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(28)" ::: "memory");  // R == 8
#pragma unroll
      for (int u = 0; u < TW; ++u) {
        const u32x4 v = *(const u32x4*)(ring + (d * TW + u) * 1024 + lane * 16);
        x ^= v[0] ^ v[1] ^ v[2] ^ v[3];
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slot is read before it is refilled
    }
  }
  sink[blockIdx.x * NW * 64 + threadIdx.x] = x;
}

typedef void (*Kern)(const u32x4*, long long, unsigned*);

struct Cfg {
  const char* name;
  Kern k;
  int nwg, nw;
  unsigned lds;
};

int main() {
  const long long POOL = 8LL << 29;  // 4 GiB: 8 buffers 512 MiB apart
  char* pool;
  CHECK(hipMalloc(&pool, POOL));
  CHECK(hipMemset(pool, 0x5a, POOL));
  unsigned* sink;
  CHECK(hipMalloc(&sink, 4 << 20));
  const Cfg cfgs[] = {
      {"reg 768x4 D2", reg_stream<4, 2>, 768, 4, 0},       {"reg 768x4 D3", reg_stream<4, 3>, 768, 4, 0},
      {"reg 256x8 D3", reg_stream<8, 3>, 256, 8, 0},       {"reg 512x8 D3", reg_stream<8, 3>, 512, 8, 0},
      {"reg 256x16 D3", reg_stream<16, 3>, 256, 16, 0},    {"lds 768x4 R3", lds_stream<4, 3>, 768, 4, 4 * 3 * 4096},
      {"lds 256x8 R4", lds_stream<8, 4>, 256, 8, 8 * 4 * 4096}, {"lds 256x4 R8", lds_stream<4, 8>, 256, 4, 4 * 8 * 4096},
      {"lds 512x4 R4", lds_stream<4, 4>, 512, 4, 4 * 4 * 4096}, {"lds 256x16 R2", lds_stream<16, 2>, 256, 16, 16 * 2 * 4096},
  };
  const double sizes_mb[] = {201.85, 100.66, 50.33, 33.55};
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  printf("{\"results\": [\n");
  bool first = true;
  for (double mb : sizes_mb) {
    for (const Cfg& c : cfgs) {
      // slice per workgroup: whole batches of every wave count (NW * TW KiB granularity)
      const long long tiles_total = (long long)(mb * 1e6) / 1024;
      const long long gran = (long long)c.nw * TW;
      const long long slice = std::max(gran, tiles_total / c.nwg / gran * gran);
      const double bytes = (double)slice * c.nwg * 1024;
      if (c.lds > 65536) CHECK(hipFuncSetAttribute((const void*)c.k, hipFuncAttributeMaxDynamicSharedMemorySize, c.lds));
      std::vector<float> t;
      for (int rep = 0; rep < 13; ++rep) {
        const u32x4* w = (const u32x4*)(pool + ((long long)(rep % 8) << 29));
        CHECK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(c.k, dim3(c.nwg), dim3(c.nw * 64), c.lds, 0, w, slice, sink);
        CHECK(hipGetLastError());
        CHECK(hipEventRecord(e1, 0));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (rep >= 3) t.push_back(ms);
      }
      std::sort(t.begin(), t.end());
      const double med = t[t.size() / 2] * 1e-3;
      printf("%s  {\"mb\": %.2f, \"cfg\": \"%s\", \"us\": %.2f, \"TBps\": %.3f, \"best_TBps\": %.3f}", first ? "" : ",\n",
             bytes / 1e6, c.name, med * 1e6, bytes / med / 1e12, bytes / (t[0] * 1e-3) / 1e12);
      first = false;
      fflush(stdout);
    }
  }
  printf("\n]}\n");
  CHECK(hipFree(pool));
  CHECK(hipFree(sink));
  return 0;
}
