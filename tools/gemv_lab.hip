// Decode-GEMM (M <= 16) design lab: times kernel variants on the Qwen3-8B decode shapes with
// weights rotated over > 1 GB (no Infinity-Cache reuse, as in a real 36-layer step).
// Standalone; not part of the engine.  Build + run on the GPU box:
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 -I inferd_amd/csrc tools/gemv_lab.hip -o /tmp/gemv_lab && /tmp/gemv_lab
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <utility>
#include <vector>

#include "common.h"

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

template <bool NT>
__device__ __forceinline__ bf16x8 ldw(const bf16x8* p) {
  if constexpr (NT)
    return __builtin_nontemporal_load(p);
  else
    return *p;
}

// Variant "round": WG = one 16-col tile (x S streams), NW waves, batches of TW k-tiles,
// wave w takes batches w, w+NW, ...; PIPE = issue batch i+1 before computing batch i.
template <int S, int NW, int TW, bool PIPE, bool NT>
__global__ __launch_bounds__(NW * 64) void gemv_round(const u16* __restrict__ A, int lda, const u16* __restrict__ Wp,
                                                      int KT, int n_tiles, float* __restrict__ C, int M) {
  __shared__ f32x4 red[NW][S * 64];
  const int nt = blockIdx.x;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const bf16x8* w0 = (const bf16x8*)(Wp + (int64_t)nt * KT * 512) + lane;
  const bf16x8* w1 = (const bf16x8*)(Wp + (int64_t)(nt + n_tiles) * KT * 512) + lane;
  int row = lane & 15;
  row = row < M ? row : M - 1;
  const u16* a = A + (int64_t)row * lda + 8 * (lane >> 4);
  f32x4 acc[S];
#pragma unroll
  for (int s = 0; s < S; ++s) acc[s] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nb = (KT + TW - 1) / TW;  // batches (KT % TW == 0 assumed)
  int b = wave;
  if (!PIPE) {
    for (; b < nb; b += NW) {
      bf16x8 wv[S][TW], av[TW];
#pragma unroll
      for (int u = 0; u < TW; ++u) {
        wv[0][u] = ldw<NT>(w0 + (b * TW + u) * 64);
        if constexpr (S == 2) wv[1][u] = ldw<NT>(w1 + (b * TW + u) * 64);
      }
#pragma unroll
      for (int u = 0; u < TW; ++u) av[u] = *(const bf16x8*)(a + (b * TW + u) * 32);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < TW; ++u)
#pragma unroll
        for (int s = 0; s < S; ++s) acc[s] = mfma16(av[u], wv[s][u], acc[s]);
    }
  } else {
    bf16x8 wa[S][TW], aa[TW], wb[S][TW], ab[TW];
#define ISSUE(WV, AV, BB)                                                   \
  {                                                                         \
    const int bc_ = (BB);                                                   \
    _Pragma("unroll") for (int u = 0; u < TW; ++u) {                        \
      WV[0][u] = ldw<NT>(w0 + (bc_ * TW + u) * 64);                         \
      if constexpr (S == 2) WV[1][u] = ldw<NT>(w1 + (bc_ * TW + u) * 64);   \
    }                                                                       \
    _Pragma("unroll") for (int u = 0; u < TW; ++u) AV[u] = *(const bf16x8*)(a + (bc_ * TW + u) * 32); \
  }
#define COMPUTE(WV, AV)                                                     \
  _Pragma("unroll") for (int u = 0; u < TW; ++u)                            \
      _Pragma("unroll") for (int s = 0; s < S; ++s) acc[s] = mfma16(AV[u], WV[s][u], acc[s]);
    if (b < nb) {
      ISSUE(wa, aa, b);
      for (;;) {
        if (b + NW < nb) ISSUE(wb, ab, b + NW);
        __builtin_amdgcn_sched_barrier(0);
        COMPUTE(wa, aa);
        __builtin_amdgcn_sched_barrier(0);
        b += NW;
        if (b >= nb) break;
        if (b + NW < nb) ISSUE(wa, aa, b + NW);
        __builtin_amdgcn_sched_barrier(0);
        COMPUTE(wb, ab);
        __builtin_amdgcn_sched_barrier(0);
        b += NW;
        if (b >= nb) break;
      }
    }
#undef ISSUE
#undef COMPUTE
  }
#pragma unroll
  for (int s = 0; s < S; ++s) red[wave][s * 64 + lane] = acc[s];
  __syncthreads();
  if (threadIdx.x < S * 64) {
    f32x4 t = red[0][threadIdx.x];
#pragma unroll
    for (int w = 1; w < NW; ++w) t += red[w][threadIdx.x];
    const int s = threadIdx.x >> 6, ln = threadIdx.x & 63;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rr = 4 * (ln >> 4) + r;
      if (rr < M) C[(int64_t)rr * (n_tiles * 16 * S) + s * n_tiles * 16 + nt * 16 + (ln & 15)] = t[r];
    }
  }
}

// Variant "ring": D register stages of TW k-tiles each; batch b+(D-1)*NW is issued before
// batch b is consumed, so (D-1)*TW weight tiles per wave stay in flight during compute.
template <int S, int NW, int TW, int D, bool NT>
__global__ __launch_bounds__(NW * 64) void gemv_ring(const u16* __restrict__ A, int lda, const u16* __restrict__ Wp,
                                                     int KT, int n_tiles, float* __restrict__ C, int M) {
  __shared__ f32x4 red[NW][S * 64];
  const int nt = blockIdx.x;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const bf16x8* w0 = (const bf16x8*)(Wp + (int64_t)nt * KT * 512) + lane;
  const bf16x8* w1 = (const bf16x8*)(Wp + (int64_t)(nt + n_tiles) * KT * 512) + lane;
  int row = lane & 15;
  row = row < M ? row : M - 1;
  const u16* a = A + (int64_t)row * lda + 8 * (lane >> 4);
  f32x4 acc[S];
#pragma unroll
  for (int s = 0; s < S; ++s) acc[s] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nb = KT / TW;
  int b = wave;
  bf16x8 wv[D][S][TW], av[D][TW];
  auto issue = [&](auto stage, int bb) {
    constexpr int d = decltype(stage)::value;
#pragma unroll
    for (int u = 0; u < TW; ++u) {
      wv[d][0][u] = ldw<NT>(w0 + (bb * TW + u) * 64);
      if constexpr (S == 2) wv[d][1][u] = ldw<NT>(w1 + (bb * TW + u) * 64);
    }
#pragma unroll
    for (int u = 0; u < TW; ++u) av[d][u] = *(const bf16x8*)(a + (bb * TW + u) * 32);
  };
  auto compute = [&](auto stage) {
    constexpr int d = decltype(stage)::value;
#pragma unroll
    for (int u = 0; u < TW; ++u)
#pragma unroll
      for (int s = 0; s < S; ++s) acc[s] = mfma16(av[d][u], wv[d][s][u], acc[s]);
  };
  if (b < nb) {
    [&]<int... I>(std::integer_sequence<int, I...>) {
      ((b + I * NW < nb ? issue(std::integral_constant<int, I>{}, b + I * NW) : void()), ...);
    }(std::make_integer_sequence<int, D - 1>{});
    bool fin = false;
    while (!fin) {
      [&]<int... I>(std::integer_sequence<int, I...>) {
        auto step = [&](auto stage) {
          constexpr int d = decltype(stage)::value;
          if (fin) return;
          const int nxt = b + (D - 1) * NW;
          if (nxt < nb) issue(std::integral_constant<int, (d + D - 1) % D>{}, nxt);
          __builtin_amdgcn_sched_barrier(0);
          compute(stage);
          __builtin_amdgcn_sched_barrier(0);
          b += NW;
          if (b >= nb) fin = true;
        };
        (step(std::integral_constant<int, I>{}), ...);
      }(std::make_integer_sequence<int, D>{});
    }
  }
#pragma unroll
  for (int s = 0; s < S; ++s) red[wave][s * 64 + lane] = acc[s];
  __syncthreads();
  if (threadIdx.x < S * 64) {
    f32x4 t = red[0][threadIdx.x];
#pragma unroll
    for (int w = 1; w < NW; ++w) t += red[w][threadIdx.x];
    const int s = threadIdx.x >> 6, ln = threadIdx.x & 63;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rr = 4 * (ln >> 4) + r;
      if (rr < M) C[(int64_t)rr * (n_tiles * 16 * S) + s * n_tiles * 16 + nt * 16 + (ln & 15)] = t[r];
    }
  }
}

// Variant "old": NW waves, contiguous K range per wave, U-tile chunks (the r01 kernel).
template <int S, int NW, int U>
__global__ __launch_bounds__(NW * 64) void gemv_old(const u16* __restrict__ A, int lda, const u16* __restrict__ Wp,
                                                    int KT, int n_tiles, float* __restrict__ C, int M) {
  __shared__ f32x4 red[NW][S * 64];
  const int nt = blockIdx.x;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int kt0 = (wave * KT) / NW, kt1 = ((wave + 1) * KT) / NW;
  const bf16x8* w0 = (const bf16x8*)(Wp + (int64_t)nt * KT * 512) + lane;
  const bf16x8* w1 = (const bf16x8*)(Wp + (int64_t)(nt + n_tiles) * KT * 512) + lane;
  int row = lane & 15;
  row = row < M ? row : M - 1;
  const u16* a = A + (int64_t)row * lda + 8 * (lane >> 4);
  f32x4 acc[S];
#pragma unroll
  for (int s = 0; s < S; ++s) acc[s] = f32x4{0.f, 0.f, 0.f, 0.f};
  int kt = kt0;
  for (; kt + U <= kt1; kt += U) {
    bf16x8 wv[S][U], av[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      wv[0][u] = w0[(kt + u) * 64];
      if constexpr (S == 2) wv[1][u] = w1[(kt + u) * 64];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) av[u] = *(const bf16x8*)(a + (kt + u) * 32);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int s = 0; s < S; ++s) acc[s] = mfma16(av[u], wv[s][u], acc[s]);
  }
  for (; kt < kt1; ++kt) {
    const bf16x8 av = *(const bf16x8*)(a + kt * 32);
    acc[0] = mfma16(av, w0[kt * 64], acc[0]);
    if constexpr (S == 2) acc[1] = mfma16(av, w1[kt * 64], acc[1]);
  }
#pragma unroll
  for (int s = 0; s < S; ++s) red[wave][s * 64 + lane] = acc[s];
  __syncthreads();
  if (threadIdx.x < S * 64) {
    f32x4 t = red[0][threadIdx.x];
#pragma unroll
    for (int w = 1; w < NW; ++w) t += red[w][threadIdx.x];
    const int s = threadIdx.x >> 6, ln = threadIdx.x & 63;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rr = 4 * (ln >> 4) + r;
      if (rr < M) C[(int64_t)rr * (n_tiles * 16 * S) + s * n_tiles * 16 + nt * 16 + (ln & 15)] = t[r];
    }
  }
}

__global__ void fill_kernel(u16* p, size_t n, uint64_t seed) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint64_t r = splitmix64(seed ^ i);
    float f = ((float)(r & 0xFFFF) / 65536.0f - 0.5f) * 0.1f;
    p[i] = f2bf(f);
  }
}

typedef void (*KFn)(const u16*, int, const u16*, int, int, float*, int);
struct Var {
  const char* name;
  KFn fn;
  int nw;
  int s;
};

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 16;
  struct Shape {
    const char* name;
    int N, K, S;
  } shapes[] = {{"qkv", 6144, 4096, 1}, {"o", 4096, 4096, 1}, {"gateup", 12288, 4096, 2}, {"down", 4096, 12288, 1}};
  std::vector<Var> v1 = {
      {"old nw8 u8", gemv_old<1, 8, 8>, 8, 1},
      {"pipe nw8 tw4 nt", gemv_round<1, 8, 4, true, true>, 8, 1},
      {"ring nw8 tw4 d2 nt", gemv_ring<1, 8, 4, 2, true>, 8, 1},
      {"ring nw8 tw4 d3 nt", gemv_ring<1, 8, 4, 3, true>, 8, 1},
      {"ring nw8 tw2 d3 nt", gemv_ring<1, 8, 2, 3, true>, 8, 1},
      {"ring nw8 tw2 d4 nt", gemv_ring<1, 8, 2, 4, true>, 8, 1},
      {"ring nw8 tw2 d6 nt", gemv_ring<1, 8, 2, 6, true>, 8, 1},
      {"ring nw4 tw4 d2 nt", gemv_ring<1, 4, 4, 2, true>, 4, 1},
      {"ring nw4 tw4 d3 nt", gemv_ring<1, 4, 4, 3, true>, 4, 1},
      {"ring nw4 tw4 d4 nt", gemv_ring<1, 4, 4, 4, true>, 4, 1},
      {"ring nw4 tw8 d2 nt", gemv_ring<1, 4, 8, 2, true>, 4, 1},
      {"ring nw16 tw2 d3 nt", gemv_ring<1, 16, 2, 3, true>, 16, 1},
      {"ring nw16 tw4 d2 nt", gemv_ring<1, 16, 4, 2, true>, 16, 1},
      {"ring nw8 tw4 d3", gemv_ring<1, 8, 4, 3, false>, 8, 1},
  };
  std::vector<Var> v2 = {
      {"old nw8 u8", gemv_old<2, 8, 8>, 8, 2},
      {"pipe nw4 tw4 nt", gemv_round<2, 4, 4, true, true>, 4, 2},
      {"ring nw4 tw4 d2 nt", gemv_ring<2, 4, 4, 2, true>, 4, 2},
      {"ring nw4 tw4 d3 nt", gemv_ring<2, 4, 4, 3, true>, 4, 2},
      {"ring nw4 tw2 d3 nt", gemv_ring<2, 4, 2, 3, true>, 4, 2},
      {"ring nw4 tw2 d4 nt", gemv_ring<2, 4, 2, 4, true>, 4, 2},
      {"ring nw8 tw2 d3 nt", gemv_ring<2, 8, 2, 3, true>, 8, 2},
      {"ring nw8 tw2 d2 nt", gemv_ring<2, 8, 2, 2, true>, 8, 2},
      {"ring nw8 tw4 d2 nt", gemv_ring<2, 8, 4, 2, true>, 8, 2},
      {"ring nw16 tw2 d2 nt", gemv_ring<2, 16, 2, 2, true>, 16, 2},
  };
  u16* A;
  float *C, *Cref;
  CHECK(hipMalloc(&A, 64 * 16384 * 2));
  CHECK(hipMalloc(&C, 64 * 32768 * 4));
  CHECK(hipMalloc(&Cref, 64 * 32768 * 4));
  hipLaunchKernelGGL(fill_kernel, dim3(1024), dim3(256), 0, 0, A, (size_t)64 * 16384, 7ull);
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (auto& sh : shapes) {
    const size_t wbytes = (size_t)sh.N * sh.S * sh.K * 2;
    const int R = (int)((1536ull << 20) / wbytes) + 1;  // copies rotated: > 1.5 GB
    std::vector<u16*> W(R);
    for (int r = 0; r < R; ++r) {
      CHECK(hipMalloc(&W[r], wbytes));
      hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, W[r], wbytes / 2, 100ull + r);
    }
    CHECK(hipDeviceSynchronize());
    const int KT = sh.K / 32, n_tiles = sh.N / 16;
    auto& vars = sh.S == 2 ? v2 : v1;
    printf("== %s N=%d K=%d S=%d M=%d  %.1f MB x %d copies\n", sh.name, sh.N, sh.K, sh.S, M, wbytes / 1e6, R);
    bool first = true;
    for (auto& v : vars) {
      const size_t outn = (size_t)M * sh.N * sh.S;
      hipLaunchKernelGGL(v.fn, dim3(n_tiles), dim3(v.nw * 64), 0, 0, A, 16384, W[0], KT, n_tiles, C, M);
      CHECK(hipDeviceSynchronize());
      if (first) {
        CHECK(hipMemcpy(Cref, C, outn * 4, hipMemcpyDeviceToDevice));
        first = false;
      }
      std::vector<float> h(outn), hr(outn);
      CHECK(hipMemcpy(h.data(), C, outn * 4, hipMemcpyDeviceToHost));
      CHECK(hipMemcpy(hr.data(), Cref, outn * 4, hipMemcpyDeviceToHost));
      double maxd = 0;
      for (size_t i = 0; i < outn; ++i) {
        double d = fabs((double)h[i] - hr[i]);
        maxd = d > maxd ? d : maxd;
      }
      const int iters = 4 * R;
      for (int it = 0; it < R; ++it)
        hipLaunchKernelGGL(v.fn, dim3(n_tiles), dim3(v.nw * 64), 0, 0, A, 16384, W[it % R], KT, n_tiles, C, M);
      CHECK(hipEventRecord(e0));
      for (int it = 0; it < iters; ++it)
        hipLaunchKernelGGL(v.fn, dim3(n_tiles), dim3(v.nw * 64), 0, 0, A, 16384, W[it % R], KT, n_tiles, C, M);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      const double us = ms * 1e3 / iters;
      printf("  %-22s %8.2f us  %7.0f GB/s  maxdiff %.2e\n", v.name, us, wbytes / (us * 1e-6) / 1e9, maxd);
    }
    for (auto p : W) CHECK(hipFree(p));
  }
  return 0;
}
