// bf16 MFMA projections of the Qwen3 layer: q/k/v (fused), o (+residual), gate/up
// (fused, SwiGLU epilogue), down (+residual), and the last span's lm_head (+argmax).
// Reference ops: nn.Linear in Qwen3Attention / Qwen3MLP
// (models/qwen3/server/qwen3_server_module.py:103-120, :33-40) and LastStage.lm_head
// (petals/partitioned_models.py:96) -- bf16 inputs, fp32 accumulate, one output rounding.
//
// Two kernels, both on v_mfma_f32_16x16x32_bf16 with weights in the fragment-packed
// layout of common.h:
//  * gemm_skinny: M <= 64 rows (decode).  HBM-bound weight stream: one workgroup per
//    16-column tile, the K range split across its waves, every weight tile fetched
//    exactly once straight into VGPRs (1 KiB dwordx4 per wave-instruction), partial
//    sums reduced through LDS, epilogue fused.
//  * gemm_tiled: M > 64 rows (prefill).  128x128x64 block tile, 4 waves (2x2, 64x64
//    each), A and B staged through double-buffered LDS with global_load_lds (A
//    XOR-swizzled on the source address, B already fragment-ordered), 32 MFMA per
//    wave per K-step.
#include "common.h"
#include "kernels.h"

__device__ __forceinline__ float silu_f(float g) { return g / (1.0f + expf(-g)); }

// ============================================================ skinny (decode) kernel
template <int MT, int NW, int EPI>
__global__ __launch_bounds__(NW * 64) void gemm_skinny_kernel(
    const u16* __restrict__ A, int64_t lda, const u16* __restrict__ Wp, int KT, int n_tiles,
    u16* __restrict__ C, int64_t ldc, const u16* __restrict__ R, int64_t ldr, int M,
    unsigned long long* __restrict__ partial) {
  constexpr int S = (EPI == EPI_SILU) ? 2 : 1;
  __shared__ float red[NW * S * MT * 256];
  const int nt = blockIdx.x;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int kt0 = (wave * KT) / NW, kt1 = ((wave + 1) * KT) / NW;
  const bf16x8* w0 = (const bf16x8*)(Wp + (int64_t)nt * KT * 512) + lane;
  const bf16x8* w1 = (const bf16x8*)(Wp + (int64_t)(nt + n_tiles) * KT * 512) + lane;
  const u16* a[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    int row = mt * 16 + (lane & 15);
    row = row < M ? row : M - 1;  // rows >= M compute garbage that is never stored
    a[mt] = A + (int64_t)row * lda + 8 * (lane >> 4);
  }
  f32x4 acc[S][MT];
#pragma unroll
  for (int s = 0; s < S; ++s)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[s][mt] = f32x4{0.f, 0.f, 0.f, 0.f};

  constexpr int U = (MT <= 2) ? 8 : 4;
  int kt = kt0;
  for (; kt + U <= kt1; kt += U) {
    bf16x8 wv[S][U];
    bf16x8 av[U][MT];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      wv[0][u] = w0[(kt + u) * 64];
      if constexpr (S == 2) wv[1][u] = w1[(kt + u) * 64];
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) av[u][mt] = *(const bf16x8*)(a[mt] + (kt + u) * 32);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int s = 0; s < S; ++s)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) acc[s][mt] = mfma16(av[u][mt], wv[s][u], acc[s][mt]);
  }
  for (; kt < kt1; ++kt) {
    bf16x8 wv0 = w0[kt * 64];
    bf16x8 wv1;
    if constexpr (S == 2) wv1 = w1[kt * 64];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      bf16x8 av = *(const bf16x8*)(a[mt] + kt * 32);
      acc[0][mt] = mfma16(av, wv0, acc[0][mt]);
      if constexpr (S == 2) acc[1][mt] = mfma16(av, wv1, acc[1][mt]);
    }
  }
  // cross-wave reduction: red[wave][s][mt][r][lane]
#pragma unroll
  for (int s = 0; s < S; ++s)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[(((wave * S + s) * MT + mt) * 4 + r) * 64 + lane] = acc[s][mt][r];
  __syncthreads();
  for (int idx = threadIdx.x; idx < MT * 256; idx += NW * 64) {
    const int mt = idx >> 8, r = (idx >> 6) & 3, ln = idx & 63;
    float v[S];
#pragma unroll
    for (int s = 0; s < S; ++s) {
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) t += red[(((w * S + s) * MT + mt) * 4 + r) * 64 + ln];
      v[s] = t;
    }
    const int row = mt * 16 + 4 * (ln >> 4) + r;
    const int col = nt * 16 + (ln & 15);
    if constexpr (EPI == EPI_ARGMAX) {
      float lv = rbf(v[0]);
      unsigned long long key = ((unsigned long long)float_key(lv) << 32) | (0xFFFFFFFFu - (uint32_t)col);
      // max over the 16 columns held by lanes with the same (ln >> 4)
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) {
        unsigned long long other = __shfl_xor(key, o, 16);
        key = other > key ? other : key;
      }
      if (row < M) {
        if ((ln & 15) == 0) partial[(int64_t)nt * M + row] = key;
        if (C) C[(int64_t)row * ldc + col] = f2bf(lv);
      }
    } else if (row < M) {
      float o;
      if constexpr (EPI == EPI_NONE) {
        o = v[0];
      } else if constexpr (EPI == EPI_RESID) {
        o = rbf(v[0]) + bf2f(R[(int64_t)row * ldr + col]);
      } else {  // EPI_SILU
        o = rbf(silu_f(rbf(v[0]))) * rbf(v[1]);
      }
      C[(int64_t)row * ldc + col] = f2bf(o);
    }
  }
}

template <int MT, int EPI>
static void skinny_dispatch(const u16* A, int64_t lda, const u16* Wp, int KT, int n_tiles, u16* C,
                            int64_t ldc, const u16* R, int64_t ldr, int M,
                            unsigned long long* partial, hipStream_t s) {
  constexpr int NW = 8;
  hipLaunchKernelGGL((gemm_skinny_kernel<MT, NW, EPI>), dim3(n_tiles), dim3(NW * 64), 0, s, A, lda,
                     Wp, KT, n_tiles, C, ldc, R, ldr, M, partial);
}

template <int EPI>
static void skinny_mt(const u16* A, int64_t lda, const u16* Wp, int KT, int n_tiles, u16* C,
                      int64_t ldc, const u16* R, int64_t ldr, int M, unsigned long long* partial,
                      hipStream_t s) {
  if (M <= 16)
    skinny_dispatch<1, EPI>(A, lda, Wp, KT, n_tiles, C, ldc, R, ldr, M, partial, s);
  else if (M <= 32)
    skinny_dispatch<2, EPI>(A, lda, Wp, KT, n_tiles, C, ldc, R, ldr, M, partial, s);
  else if (M <= 48)
    skinny_dispatch<3, EPI>(A, lda, Wp, KT, n_tiles, C, ldc, R, ldr, M, partial, s);
  else
    skinny_dispatch<4, EPI>(A, lda, Wp, KT, n_tiles, C, ldc, R, ldr, M, partial, s);
}

// ============================================================ tiled (prefill) kernel
#define TBM 128
#define TBN 128
#define TBK 64

template <int EPI>
__global__ __launch_bounds__(256) void gemm_tiled_kernel(
    const u16* __restrict__ A, int64_t lda, const u16* __restrict__ Wp, int KT, int n_tiles_w,
    u16* __restrict__ C, int64_t ldc, const u16* __restrict__ R, int64_t ldr, int M) {
  // LDS: 2 buffers x (A 16 KiB + B 16 KiB), one array (guide §5 trap 4a)
  __shared__ __attribute__((aligned(16))) char lds[2 * 32768];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wr = wave >> 1, wc = wave & 1;
  const int m0 = blockIdx.y * TBM;
  // output-column block: EPI_SILU blocks are 64 wide ([gate 64 | up 64] in the B tile)
  const int ncols = (EPI == EPI_SILU) ? 64 : 128;
  const int n0 = blockIdx.x * ncols;
  const int nsteps = KT / 2;

  // --- staging assignment: each wave issues 4 A pieces and 4 B pieces per K-step.
  // A piece q (0..15): rows 8q..8q+7 x 64 k; lane i -> row 8q + i/8, lds slot i%8 holds
  // source chunk (i%8) ^ ((row >> 1) & 7)  (XOR swizzle on the source address).
  const u16* a_src[4];
  int a_lds[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    int q = wave * 4 + p;
    int r = 8 * q + (lane >> 3);
    int grow = m0 + r;
    grow = grow < M ? grow : M - 1;
    int chunk = (lane & 7) ^ ((r >> 1) & 7);
    a_src[p] = A + (int64_t)grow * lda + chunk * 8;
    a_lds[p] = q * 1024;
  }
  // B piece q (0..15): local n-tile j = q/2, k-tile kk = q%2 -> one packed 1 KiB tile
  const u16* b_src[4];
  int b_lds[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    int q = wave * 4 + p;
    int j = q >> 1, kk = q & 1;
    int gnt;
    if (EPI == EPI_SILU)
      gnt = (j < 4) ? (n0 / 16 + j) : (n_tiles_w / 2 + n0 / 16 + (j - 4));
    else
      gnt = n0 / 16 + j;
    b_src[p] = Wp + ((int64_t)gnt * KT + kk) * 512 + lane * 8;
    b_lds[p] = 16384 + q * 1024;
  }

  auto stage = [&](int buf, int step) {
    char* base = lds + buf * 32768;
#pragma unroll
    for (int p = 0; p < 4; ++p)
      __builtin_amdgcn_global_load_lds((const void*)(a_src[p] + step * TBK), (void*)(base + a_lds[p]), 16, 0, 0);
#pragma unroll
    for (int p = 0; p < 4; ++p)
      __builtin_amdgcn_global_load_lds((const void*)(b_src[p] + (int64_t)step * 2 * 512), (void*)(base + b_lds[p]), 16, 0, 0);
  };

  // local n-tiles this wave consumes
  int bj[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    if (EPI == EPI_SILU)
      bj[t] = (t < 2) ? (wc * 2 + t) : (4 + wc * 2 + (t - 2));
    else
      bj[t] = wc * 4 + t;
  }

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  stage(0, 0);
  __syncthreads();
  for (int t = 0; t < nsteps; ++t) {
    const int cur = t & 1;
    if (t + 1 < nsteps) stage(cur ^ 1, t + 1);
    const char* base = lds + cur * 32768;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        int r = wr * 64 + mt * 16 + (lane & 15);
        int c = kk * 4 + (lane >> 4);
        af[mt] = *(const bf16x8*)(base + r * 128 + 16 * (c ^ ((r >> 1) & 7)));
      }
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
        bfr[nt] = *(const bf16x8*)(base + 16384 + (bj[nt] * 2 + kk) * 1024 + lane * 16);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) acc[mt][nt] = mfma16(af[mt], bfr[nt], acc[mt][nt]);
    }
    __syncthreads();
  }

  // epilogue
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = m0 + wr * 64 + mt * 16 + 4 * (lane >> 4) + r;
      if (row >= M) continue;
      if constexpr (EPI == EPI_SILU) {
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          const int col = n0 + wc * 32 + nt * 16 + (lane & 15);
          float g = rbf(acc[mt][nt][r]);
          float u = rbf(acc[mt][nt + 2][r]);
          C[(int64_t)row * ldc + col] = f2bf(rbf(silu_f(g)) * u);
        }
      } else {
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
          const int col = n0 + wc * 64 + nt * 16 + (lane & 15);
          float o = acc[mt][nt][r];
          if constexpr (EPI == EPI_RESID) o = rbf(o) + bf2f(R[(int64_t)row * ldr + col]);
          C[(int64_t)row * ldc + col] = f2bf(o);
        }
      }
    }
  }
}

// ============================================================ dispatch
void launch_gemm(const u16* A, int64_t lda, const u16* Wp, int M, int N, int K, u16* C,
                 int64_t ldc, const u16* R, int64_t ldr, int epi, unsigned long long* partial,
                 hipStream_t s) {
  const int KT = K / 32;
  const int n_tiles = N / 16;  // output tiles of 16 columns
  const bool tiled_ok = (M > 64) && (K % TBK == 0) &&
                        ((epi == EPI_SILU) ? (N % 64 == 0) : (N % TBN == 0)) && epi != EPI_ARGMAX;
  if (tiled_ok) {
    const int ncols = (epi == EPI_SILU) ? 64 : 128;
    dim3 g(N / ncols, (M + TBM - 1) / TBM);
    const int ntw = (epi == EPI_SILU) ? 2 * n_tiles : n_tiles;
    switch (epi) {
      case EPI_NONE:
        hipLaunchKernelGGL(gemm_tiled_kernel<EPI_NONE>, g, dim3(256), 0, s, A, lda, Wp, KT, ntw, C, ldc, R, ldr, M);
        break;
      case EPI_RESID:
        hipLaunchKernelGGL(gemm_tiled_kernel<EPI_RESID>, g, dim3(256), 0, s, A, lda, Wp, KT, ntw, C, ldc, R, ldr, M);
        break;
      default:
        hipLaunchKernelGGL(gemm_tiled_kernel<EPI_SILU>, g, dim3(256), 0, s, A, lda, Wp, KT, ntw, C, ldc, R, ldr, M);
        break;
    }
    return;
  }
  // skinny path, 64-row slabs (M > 64 only when the tiled shape constraints fail)
  for (int m0 = 0; m0 < M; m0 += 64) {
    const int mm = (M - m0) < 64 ? (M - m0) : 64;
    const u16* Am = A + (int64_t)m0 * lda;
    u16* Cm = C ? C + (int64_t)m0 * ldc : nullptr;
    const u16* Rm = R ? R + (int64_t)m0 * ldr : nullptr;
    switch (epi) {
      case EPI_NONE: skinny_mt<EPI_NONE>(Am, lda, Wp, KT, n_tiles, Cm, ldc, Rm, ldr, mm, partial, s); break;
      case EPI_RESID: skinny_mt<EPI_RESID>(Am, lda, Wp, KT, n_tiles, Cm, ldc, Rm, ldr, mm, partial, s); break;
      case EPI_SILU: skinny_mt<EPI_SILU>(Am, lda, Wp, KT, n_tiles, Cm, ldc, Rm, ldr, mm, partial, s); break;
      default: skinny_mt<EPI_ARGMAX>(Am, lda, Wp, KT, n_tiles, Cm, ldc, Rm, ldr, mm, partial, s); break;
    }
    if (epi == EPI_ARGMAX) break;  // argmax requires M <= 64 (checked by the caller)
  }
}

// per-row max over n_tiles partial keys -> token id (lowest index among equal maxima)
__global__ __launch_bounds__(256) void argmax_reduce_kernel(const unsigned long long* __restrict__ partial,
                                                            int n_tiles, int M, int32_t* __restrict__ ids) {
  __shared__ unsigned long long red[4];
  const int row = blockIdx.x;
  unsigned long long best = 0;
  for (int t = threadIdx.x; t < n_tiles; t += 256) {
    unsigned long long k = partial[(int64_t)t * M + row];
    best = k > best ? k : best;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    unsigned long long other = __shfl_xor(best, o);
    best = other > best ? other : best;
  }
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = best;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long b = red[0];
    for (int w = 1; w < 4; ++w) b = red[w] > b ? red[w] : b;
    ids[row] = (int32_t)(0xFFFFFFFFu - (uint32_t)(b & 0xFFFFFFFFull));
  }
}

void launch_argmax_reduce(const unsigned long long* partial, int n_tiles, int M, int32_t* ids,
                          hipStream_t s) {
  hipLaunchKernelGGL(argmax_reduce_kernel, dim3(M), dim3(256), 0, s, partial, n_tiles, M, ids);
}
