// bf16 MFMA projections of the Qwen3 layer: q/k/v (fused), o (+residual), gate/up
// (fused, SwiGLU epilogue), down (+residual), and the last span's lm_head (+argmax).
// Reference ops: nn.Linear in Qwen3Attention / Qwen3MLP
// (models/qwen3/server/qwen3_server_module.py:103-120, :33-40) and LastStage.lm_head
// (petals/partitioned_models.py:96) -- bf16 inputs, fp32 accumulate, one output rounding.
//
// Kernels on v_mfma_f32_16x16x32_bf16 with weights in the fragment-packed layout of
// common.h:
//  * gemm_decode: M <= 64 rows.  HBM-bound weight stream (GEMV-like).  Workgroup = NW
//    waves = one 16-column output tile (x S streams: gate and up for the SwiGLU GEMM) over
//    the whole K range.  The K tiles are cut into batches of TW (1 KiB weight tiles + the
//    matching activation fragments, straight into VGPRs); wave w takes batches w, w+NW, ...
//    through a D-stage register ring: batch i+D-1 is issued before batch i is consumed, so
//    (D-1)*TW weight tiles per wave stay in flight across the MFMAs (weights loaded
//    non-temporal: each byte is read once per step).  The NW partial accumulators reduce
//    through LDS; the epilogue (residual add / SwiGLU / argmax keys) is fused.  No split-K:
//    measured on the box, every in-launch K split cost more than the balance it bought.
//  * gemm_tiled / gemm_tiled256: M > 64 rows (prefill).  128x128 (4 waves) or 256x256
//    (8 waves) block tiles, A and B staged through double-buffered LDS with
//    global_load_lds (A XOR-swizzled on the source address, B already fragment-ordered).
#include <stdlib.h>

#include <utility>

#include "common.h"
#include "kernels.h"

__device__ __forceinline__ float silu_f(float g) { return g / (1.0f + expf(-g)); }

// ============================================================ decode (M <= 64) kernel
struct DecodeArgs {
  const u16* A;
  int64_t lda;
  const u16* Wp;
  int KT, n_tiles, M;
  u16* C;
  int64_t ldc;
  const u16* R;
  int64_t ldr;
  unsigned long long* keys;  // EPI_ARGMAX partial keys [M][n_tiles]
  float eps;                 // NORM: RMSNorm epsilon
  // EPI_PARTIAL (K split over gridDim.y slices, reduced by the consumer): slice y covers
  // k-tiles [y * KT / gridDim.y, (y + 1) * KT / gridDim.y); it writes its fp32 accumulator
  // to part[y][row][col] (row stride ldp) and, with NORM, its rows' sums of squares to
  // ssq[y][row] -- both unscaled.
  float* part;
  int64_t ldp;
  float* ssq;
};

template <int MT, int S, int NW, int TW, int D, int EPI, bool NORM>
__global__ __launch_bounds__(NW * 64) void gemm_decode_kernel(DecodeArgs g) {
  constexpr int NV = S * MT * 64;  // f32x4 values of one workgroup result
  __shared__ f32x4 red[NW][NV];
  __shared__ float sm_ss[NORM ? NW : 1][MT * 16];
  const int M = g.M;
  const int nt = blockIdx.x;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  // K range of this workgroup (all of K unless EPI_PARTIAL splits it over gridDim.y)
  const int kt0 = (EPI == EPI_PARTIAL) ? (int)blockIdx.y * (g.KT / (int)gridDim.y) : 0;
  const int KT = (EPI == EPI_PARTIAL) ? g.KT / (int)gridDim.y : g.KT;
  const bf16x8* w0 = (const bf16x8*)(g.Wp + ((int64_t)nt * g.KT + kt0) * 512) + lane;
  const bf16x8* w1 = (const bf16x8*)(g.Wp + ((int64_t)(nt + g.n_tiles) * g.KT + kt0) * 512) + lane;
  const u16* a[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    int row = mt * 16 + (lane & 15);
    row = row < M ? row : M - 1;  // rows >= M compute garbage that is never stored
    a[mt] = g.A + (int64_t)row * g.lda + 8 * (lane >> 4) + kt0 * 32;
  }
  f32x4 acc[S][MT];
#pragma unroll
  for (int s = 0; s < S; ++s)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[s][mt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float ssq[MT];  // NORM: this lane's share of sum(x^2) of row mt*16 + (lane & 15)
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) ssq[mt] = 0.f;

  const int nb = KT / TW;  // batches (the dispatcher guarantees KT % TW == 0)
  int b = wave;
  bf16x8 wv[D][S][TW], av[D][TW][MT];
  auto issue = [&](auto stage, int bb) {
    constexpr int d = decltype(stage)::value;
#pragma unroll
    for (int u = 0; u < TW; ++u) {
      wv[d][0][u] = __builtin_nontemporal_load(w0 + (bb * TW + u) * 64);
      if constexpr (S == 2) wv[d][1][u] = __builtin_nontemporal_load(w1 + (bb * TW + u) * 64);
    }
#pragma unroll
    for (int u = 0; u < TW; ++u)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) av[d][u][mt] = *(const bf16x8*)(a[mt] + (bb * TW + u) * 32);
  };
  if (b < nb) {
    // prologue: stages 0..D-2
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
          // keep the issued loads ahead of the MFMAs (the scheduler would otherwise
          // interleave them to save registers, leaving few loads in flight)
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int u = 0; u < TW; ++u)
#pragma unroll
            for (int s = 0; s < S; ++s)
#pragma unroll
              for (int mt = 0; mt < MT; ++mt) acc[s][mt] = mfma16(av[d][u][mt], wv[d][s][u], acc[s][mt]);
          if constexpr (NORM) {
#pragma unroll
            for (int u = 0; u < TW; ++u)
#pragma unroll
              for (int mt = 0; mt < MT; ++mt) {
                const u16x8 xv = __builtin_bit_cast(u16x8, av[d][u][mt]);
#pragma unroll
                for (int j = 0; j < 8; ++j) ssq[mt] = fmaf(bf2f(xv[j]), bf2f(xv[j]), ssq[mt]);
              }
          }
          __builtin_amdgcn_sched_barrier(0);
          b += NW;
          if (b >= nb) fin = true;
        };
        (step(std::integral_constant<int, I>{}), ...);
      }(std::make_integer_sequence<int, D>{});
    }
  }
#pragma unroll
  for (int s = 0; s < S; ++s)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) red[wave][(s * MT + mt) * 64 + lane] = acc[s][mt];
  if constexpr (NORM) {
    // lanes l, l^16, l^32, l^48 hold the four k-quarters of row (l & 15)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      float t = ssq[mt];
      t += __shfl_xor(t, 16);
      t += __shfl_xor(t, 32);
      if (lane < 16) sm_ss[wave][mt * 16 + lane] = t;
    }
  }
  __syncthreads();
  // thread p < MT*64 owns (mt, lane ln) of every stream s: rows mt*16 + 4*(ln>>4) + r, col ln&15
  const int p = threadIdx.x;
  if (p >= MT * 64) return;
  f32x4 v[S];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int q = s * MT * 64 + p;
    f32x4 t = red[0][q];
#pragma unroll
    for (int w = 1; w < NW; ++w) t += red[w][q];
    v[s] = t;
  }
  const int mt = p >> 6, ln = p & 63;
  const int col = nt * 16 + (ln & 15);
  if constexpr (EPI == EPI_PARTIAL) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = mt * 16 + 4 * (ln >> 4) + r;
      if (row >= M) continue;
      g.part[((int64_t)blockIdx.y * M + row) * g.ldp + col] = v[0][r];
      if constexpr (NORM) {
        if (nt == 0 && (ln & 15) == 0) {
          float t = 0.f;
#pragma unroll
          for (int w = 0; w < NW; ++w) t += sm_ss[w][row];
          g.ssq[blockIdx.y * M + row] = t;
        }
      }
    }
    return;
  }
  if constexpr (NORM) {
    // folded RMSNorm: out = rsqrt(mean(x^2) + eps) * (x @ (W * w)^T)   
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rr = mt * 16 + 4 * (ln >> 4) + r;
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) t += sm_ss[w][rr];
      const float inv = 1.0f / sqrtf(t / (float)(g.KT * 32) + g.eps);
#pragma unroll
      for (int s = 0; s < S; ++s) v[s][r] *= inv;
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = mt * 16 + 4 * (ln >> 4) + r;
    if constexpr (EPI == EPI_ARGMAX) {
      const float lv = rbf(v[0][r]);
      unsigned long long key = ((unsigned long long)float_key(lv) << 32) | (0xFFFFFFFFu - (uint32_t)col);
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) {
        const unsigned long long other = __shfl_xor(key, o, 16);
        key = other > key ? other : key;
      }
      if (row < M) {
        if ((ln & 15) == 0) g.keys[(int64_t)row * g.n_tiles + nt] = key;  // [M][n_tiles]
        if (g.C) g.C[(int64_t)row * g.ldc + col] = f2bf(lv);
      }
    } else if (row < M) {
      float o;
      if constexpr (EPI == EPI_NONE) {
        o = v[0][r];
      } else if constexpr (EPI == EPI_RESID) {
        o = rbf(v[0][r]) + bf2f(g.R[(int64_t)row * g.ldr + col]);
      } else if constexpr (EPI == EPI_SILU) {
        o = rbf(silu_f(rbf(v[0][r]))) * rbf(v[S - 1][r]);
      } else {
        o = 0.f;  // EPI_PARTIAL returns above
      }
      g.C[(int64_t)row * g.ldc + col] = f2bf(o);
    }
  }
}

// ring shape per (row tiles, streams): tuned on the Qwen3-8B decode shapes (tools/gemv_lab.hip)
template <int MT, int S>
struct DecodeCfg {
  static constexpr int NW = S == 1 ? 8 : 4;
  static constexpr int TW = (MT <= 2) ? 4 : 2;
  static constexpr int D = (S == 1 && MT == 1) ? 3 : 2;
};

template <int MT, int EPI, bool NORM>
static void decode_launch(const DecodeArgs& a, hipStream_t s) {
  constexpr int S = (EPI == EPI_SILU) ? 2 : 1;
  using C = DecodeCfg<MT, S>;
  if (a.KT % C::TW == 0)
    hipLaunchKernelGGL((gemm_decode_kernel<MT, S, C::NW, C::TW, C::D, EPI, NORM>), dim3(a.n_tiles),
                       dim3(C::NW * 64), 0, s, a);
  else  // odd K/32 (single-op API only; every Qwen3 projection has K % 128 == 0)
    hipLaunchKernelGGL((gemm_decode_kernel<MT, S, C::NW, 1, 2, EPI, NORM>), dim3(a.n_tiles), dim3(C::NW * 64), 0,
                       s, a);
}

template <int EPI, bool NORM>
static void decode_mt(const DecodeArgs& a, hipStream_t s) {
  if (a.M <= 16)
    decode_launch<1, EPI, NORM>(a, s);
  else if (a.M <= 32)
    decode_launch<2, EPI, NORM>(a, s);
  else if (a.M <= 48)
    decode_launch<3, EPI, NORM>(a, s);
  else
    decode_launch<4, EPI, NORM>(a, s);
}

// q/k/v projection of a decode step with K split over `kslices` workgroup slices and the
// reduction (+ folded-norm scale) left to the consumer (launch_attn_decode_fused): with
// NW = 4 the 384 x 2 workgroups of Qwen3-8B sit 3 per CU, every CU streaming the same bytes.
void launch_gemm_decode_partial(const u16* A, int64_t lda, const u16* Wp, int M, int N, int K, int kslices,
                                float* part, float* ssq, float eps, hipStream_t s) {
  DecodeArgs a = {};
  a.A = A;
  a.lda = lda;
  a.Wp = Wp;
  a.KT = K / 32;
  a.n_tiles = N / 16;
  a.M = M;
  a.eps = eps;
  a.part = part;
  a.ldp = N;
  a.ssq = ssq;
  hipLaunchKernelGGL((gemm_decode_kernel<1, 1, 4, 4, 3, EPI_PARTIAL, true>), dim3(N / 16, kslices), dim3(256), 0, s,
                     a);
}

// ============================================================ tiled (prefill) kernel
#define TBM 128
#define TBN 128
#define TBK 64

template <int EPI>
__global__ __launch_bounds__(256) void gemm_tiled_kernel(
    const u16* __restrict__ A, int64_t lda, const u16* __restrict__ Wp, int KT, int n_tiles_w,
    u16* __restrict__ C, int64_t ldc, const u16* __restrict__ R, int64_t ldr, int M,
    const float* __restrict__ rs) {
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
      const float sc = rs ? rs[row] : 1.0f;  // folded RMSNorm row scale
      if constexpr (EPI == EPI_SILU) {
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          const int col = n0 + wc * 32 + nt * 16 + (lane & 15);
          float g = rbf(acc[mt][nt][r] * sc);
          float u = rbf(acc[mt][nt + 2][r] * sc);
          C[(int64_t)row * ldc + col] = f2bf(rbf(silu_f(g)) * u);
        }
      } else {
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
          const int col = n0 + wc * 64 + nt * 16 + (lane & 15);
          float o = acc[mt][nt][r] * sc;
          if constexpr (EPI == EPI_RESID) o = rbf(o) + bf2f(R[(int64_t)row * ldr + col]);
          C[(int64_t)row * ldc + col] = f2bf(o);
        }
      }
    }
  }
}

// ============================================================ 256x256 tiled (large prefill)
// 256x256x64 block tile, 8 waves as 2 (M) x 4 (N), each wave 128x64 = 8x4 MFMA tiles
// (128 fp32 accumulator registers).  Per K-step the workgroup stages A (256 rows x 64 k,
// 32 KiB, source-swizzled) and B (16 n-tiles x 2 k-tiles = 32 packed 1 KiB tiles) into one
// of two 64 KiB LDS buffers with global_load_lds_dwordx4 (8 pieces per wave), overlapping
// the next step's transfer with this step's 64 MFMAs per wave.  EPI_SILU: the B tile holds
// 128 gate + 128 up columns of the same 128 outputs.
template <int EPI>
__global__ __launch_bounds__(512) void gemm_tiled256_kernel(
    const u16* __restrict__ A, int64_t lda, const u16* __restrict__ Wp, int KT, int n_tiles_w,
    u16* __restrict__ C, int64_t ldc, const u16* __restrict__ R, int64_t ldr, int M,
    const float* __restrict__ rs) {
  __shared__ __attribute__((aligned(16))) char lds[2 * 65536];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wr = wave >> 2, wc = wave & 3;
  const int m0 = blockIdx.y * 256;
  const int ncols = (EPI == EPI_SILU) ? 128 : 256;
  const int n0 = blockIdx.x * ncols;
  const int nsteps = KT / 2;
  // A pieces q = 0..31: rows 8q..8q+7; B pieces q = 0..31: local n-tile q/2, k-tile q%2
  const u16* a_src[4];
  const u16* b_src[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int q = wave * 4 + p;
    const int r = 8 * q + (lane >> 3);
    int grow = m0 + r;
    grow = grow < M ? grow : M - 1;
    const int chunk = (lane & 7) ^ ((r >> 1) & 7);
    a_src[p] = A + (int64_t)grow * lda + chunk * 8;
    const int j = q >> 1, kk = q & 1;
    int gnt;
    if (EPI == EPI_SILU)
      gnt = (j < 8) ? (n0 / 16 + j) : (n_tiles_w / 2 + n0 / 16 + (j - 8));
    else
      gnt = n0 / 16 + j;
    b_src[p] = Wp + ((int64_t)gnt * KT + kk) * 512 + lane * 8;
  }
  auto stage = [&](int buf, int step) {
    char* base = lds + buf * 65536;
#pragma unroll
    for (int p = 0; p < 4; ++p)
      __builtin_amdgcn_global_load_lds((const void*)(a_src[p] + step * 64), (void*)(base + (wave * 4 + p) * 1024),
                                       16, 0, 0);
#pragma unroll
    for (int p = 0; p < 4; ++p)
      __builtin_amdgcn_global_load_lds((const void*)(b_src[p] + (int64_t)step * 1024),
                                       (void*)(base + 32768 + (wave * 4 + p) * 1024), 16, 0, 0);
  };
  // local n-tiles of this wave (4 x 16 columns)
  int bj[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    if (EPI == EPI_SILU)
      bj[t] = (t < 2) ? (wc * 2 + t) : (8 + wc * 2 + (t - 2));
    else
      bj[t] = wc * 4 + t;
  }
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  stage(0, 0);
  __syncthreads();
  for (int t = 0; t < nsteps; ++t) {
    const int cur = t & 1;
    if (t + 1 < nsteps) stage(cur ^ 1, t + 1);
    const char* base = lds + cur * 65536;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 bfr[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) bfr[nt] = *(const bf16x8*)(base + 32768 + (bj[nt] * 2 + kk) * 1024 + lane * 16);
#pragma unroll
      for (int mt = 0; mt < 8; ++mt) {
        const int r = wr * 128 + mt * 16 + (lane & 15);
        const int c = kk * 4 + (lane >> 4);
        const bf16x8 af = *(const bf16x8*)(base + r * 128 + 16 * (c ^ ((r >> 1) & 7)));
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) acc[mt][nt] = mfma16(af, bfr[nt], acc[mt][nt]);
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int mt = 0; mt < 8; ++mt) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = m0 + wr * 128 + mt * 16 + 4 * (lane >> 4) + r;
      if (row >= M) continue;
      const float sc = rs ? rs[row] : 1.0f;  // folded RMSNorm row scale
      if constexpr (EPI == EPI_SILU) {
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          const int col = n0 + wc * 32 + nt * 16 + (lane & 15);
          const float gg = rbf(acc[mt][nt][r] * sc);
          const float uu = rbf(acc[mt][nt + 2][r] * sc);
          C[(int64_t)row * ldc + col] = f2bf(rbf(silu_f(gg)) * uu);
        }
      } else {
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
          const int col = n0 + wc * 64 + nt * 16 + (lane & 15);
          float o = acc[mt][nt][r] * sc;
          if constexpr (EPI == EPI_RESID) o = rbf(o) + bf2f(R[(int64_t)row * ldr + col]);
          C[(int64_t)row * ldc + col] = f2bf(o);
        }
      }
    }
  }
}

// ============================================================ ring-staged 256x256 (prefill)
// Same 256x256x64 block tile and 2 (M) x 4 (N) wave grid as gemm_tiled256, but the
// staging never drains (cdna_hip_programming.md §5 "Pipelining across barriers"):
//  * LDS is a ring of 10 half-tile slots of 16 KiB (the whole 160 KiB).  A K-step's
//    tile is four half-tiles consumed in this order: A0 (rows qr=0 of both wave rows),
//    B0 (columns qc=0 of every wave column), B1, A1.  Half-tile s lives in slot s % 10.
//  * One K-step = 4 phases, one per output quadrant of a wave (64 rows x 32 cols, 16
//    MFMAs): (A0,B0) (A0,B1) (A1,B1) (A1,B0).  Phase P reads its register sub-tiles,
//    issues half-tile P+6 (2 global_load_lds_dwordx4 per thread), waits with a COUNTED
//    vmcnt for the half-tile phase P+1 reads (4 half-tiles stay in flight), passes a raw
//    s_barrier, runs its 16 MFMAs at raised priority and passes a second s_barrier.
//  * Waves 4-7 run one barrier behind waves 0-3 (each SIMD holds one wave of each half),
//    so on every SIMD one wave is in its MFMA segment while its partner reads LDS.
//  * Hazards (derived in DESIGN.md §4): a slot is re-filled only >= 2 phases after its
//    last read, which bounds the look-ahead to ring - 4 = 6 half-tiles.
//  * Operands are swapped (C^T = W * A^T) so each lane's 4 accumulator registers are 4
//    consecutive output columns: the epilogue stores 8 bytes per lane.
//  * blockIdx is remapped XCD-aware (blocks sharing an XCD get consecutive tiles) and
//    grouped 8 row-blocks deep so an XCD's concurrent blocks share A rows and W columns.
#define RING_SLOTS 10

// vm_wait with a run-time count (even values 0..14; -1 = no wait); a constant argument
// folds to the single s_waitcnt
__device__ __forceinline__ void vm_wait_rt(int n) {
  switch (n) {
    case 0: vm_wait<0>(); break;
    case 2: vm_wait<2>(); break;
    case 4: vm_wait<4>(); break;
    case 6: vm_wait<6>(); break;
    case 8: vm_wait<8>(); break;
    case 10: vm_wait<10>(); break;
    case 12: vm_wait<12>(); break;
    case 14: vm_wait<14>(); break;
    default: break;
  }
}


// Tail split (SplitTail): when the tile count leaves a partial last round on an XCD
// (Qwen3-32B o/down: 640 tiles = 2.5 rounds of 256 CUs), each XCD's last `rem` tiles are
// cut into `split` K-slices so the last round is full.  Slices publish fp32 partials
// write-through (8-byte sc1 stores), take a ticket, and the last arriver of a tile polls
// the done counter, acquires, sums the partials in slice order (deterministic) and runs
// the epilogue (cdna_hip_programming.md §5 split-K, §6 Guideline 16 R1).
struct SplitTail {
  int split;            // 1 = no split
  int tiles_per_xcd;    // tiles owned by one XCD's contiguous block range
  int full_per_xcd;     // of which are computed whole
  int units_per_xcd;    // full_per_xcd + (tiles_per_xcd - full_per_xcd) * split
  float* ws;            // per split tile: split x (256 x 256) fp32 partials
  unsigned* cnt;        // [2][8 * rem] arrival tickets, done counters (zero between launches)
};

// XCD-aware tile order (bijective for any grid size): blocks that share an XCD get
// consecutive tiles, grouped GM row-blocks deep; with a tail split, each XCD's last tiles
// are cut into K-slices (SplitTail)
__device__ __forceinline__ void tile_order_v(const SplitTail& st, int grid_m, int grid_n, int orig, int nwg, int& bm,
                                             int& bn, int& slice, int& nsl, int& sidx) {
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  int tile = wg;
  if (st.split > 1) {  // grid = 8 * units_per_xcd
    const int x = wg / st.units_per_xcd, li = wg - x * st.units_per_xcd;
    if (li < st.full_per_xcd) {
      tile = x * st.tiles_per_xcd + li;
    } else {
      const int j = li - st.full_per_xcd;
      tile = x * st.tiles_per_xcd + st.full_per_xcd + j / st.split;
      slice = j % st.split;
      nsl = st.split;
      sidx = x * (st.tiles_per_xcd - st.full_per_xcd) + j / st.split;
    }
  }
  constexpr int GM = 8;
  const int group = tile / (GM * grid_n);
  const int first_m = group * GM;
  const int gsz = min(grid_m - first_m, GM);
  const int in = tile - group * GM * grid_n;
  bm = first_m + in % gsz;
  bn = in / gsz;
}

__device__ __forceinline__ void tile_order(const SplitTail& st, int grid_m, int grid_n, int& bm, int& bn,
                                           int& slice, int& nsl, int& sidx) {
  tile_order_v(st, grid_m, grid_n, blockIdx.x, gridDim.x, bm, bn, slice, nsl, sidx);
}

template <int EPI, bool KEEPB>
__global__ __launch_bounds__(512, 1) void gemm_ring256_kernel(
    const u16* __restrict__ A, int64_t lda, const u16* __restrict__ Wp, int KT, int n_tiles_w,
    u16* __restrict__ C, int64_t ldc, const u16* __restrict__ R, int64_t ldr, int M,
    const float* __restrict__ rs, int grid_m, int grid_n, SplitTail st) {
  __shared__ __attribute__((aligned(16))) char lds[RING_SLOTS * 16384];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wr = wave >> 2, wc = wave & 3;
  int bm, bn, slice = 0, nsl = 1, sidx = 0;
  tile_order(st, grid_m, grid_n, bm, bn, slice, nsl, sidx);
  const int m0 = bm * 256;
  const int n0 = bn * ((EPI == EPI_SILU) ? 128 : 256);
  const int nK = KT / 2 / nsl;  // 64-deep K-steps of this slice
  const int S = 4 * nK;         // half-tiles
  const int k0 = slice * nK;    // first K-step

  // ---- staging sources: this wave's two 1 KiB pieces of each half-tile kind
  const u16* a_src[2][2];      // [half][piece]
  const u16* b_src[2];         // [half] (the 2 pieces are the 2 consecutive k-tiles)
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int qp = 2 * wave + p;                 // piece 0..15: image rows 8qp..8qp+7
      const int i = 8 * qp + (lane >> 3);          // image row 0..127
      int grow = m0 + (i >> 6) * 128 + h * 64 + (i & 63);
      grow = grow < M ? grow : M - 1;
      const int chunk = (lane & 7) ^ ((i >> 1) & 7);
      a_src[h][p] = A + (int64_t)grow * lda + chunk * 8 + k0 * 64;
    }
    // image n-tile nl = wave: wave column nl>>1, sub-tile nl&1
    int gnt;
    if constexpr (EPI == EPI_SILU)
      gnt = (h == 0 ? 0 : n_tiles_w / 2) + n0 / 16 + (wave >> 1) * 2 + (wave & 1);
    else
      gnt = n0 / 16 + (wave >> 1) * 4 + h * 2 + (wave & 1);
    b_src[h] = Wp + ((int64_t)gnt * KT + 2 * k0) * 512 + lane * 8;
  }
  // kind: 0 = A0, 1 = B0, 2 = B1, 3 = A1 (the consumption order within a K-step)
  auto issue = [&](int kind, int t, int slot) {
    char* base = lds + slot * 16384 + wave * 2048;
    if (kind == 0 || kind == 3) {
      const int h = kind == 0 ? 0 : 1;
      __builtin_amdgcn_global_load_lds((const void*)(a_src[h][0] + t * 64), (void*)base, 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(a_src[h][1] + t * 64), (void*)(base + 1024), 16, 0, 0);
    } else {
      const u16* src = b_src[kind - 1] + (int64_t)t * 1024;
      __builtin_amdgcn_global_load_lds((const void*)src, (void*)base, 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(src + 512), (void*)(base + 1024), 16, 0, 0);
    }
  };


  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // KEEPB: both B sub-tiles stay in registers for the whole K-step (B0 is not re-read by
  // the last quadrant), so every slot's last read is no later than its own index and the
  // look-ahead grows from ring - 4 to ring - 2 half-tiles.
  constexpr int D = KEEPB ? RING_SLOTS - 2 : RING_SLOTS - 4;
  bf16x8 areg[4][2], breg[2][2][2];  // breg[quadrant column][nt][ks]

  auto read_a = [&](int slot) {
    const char* base = lds + slot * 16384;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const int i = wr * 64 + mt * 16 + (lane & 15);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int c = ks * 4 + (lane >> 4);
        areg[mt][ks] = *(const bf16x8*)(base + i * 128 + 16 * (c ^ ((i >> 1) & 7)));
      }
    }
  };
  auto read_b = [&](auto QC, int slot) {
    constexpr int qc = decltype(QC)::value;
    const char* base = lds + slot * 16384 + lane * 16;
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) breg[qc][nt][ks] = *(const bf16x8*)(base + ((wc * 2 + nt) * 2 + ks) * 1024);
  };
  auto mfmas = [&](auto QR, auto QC) {
    constexpr int qr = decltype(QR)::value, qc = decltype(QC)::value;
    constexpr int bq = KEEPB ? qc : 0;  // without KEEPB one B register set is reused
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
          acc[qr * 4 + mt][qc * 2 + nt] = mfma16(breg[bq][nt][ks], areg[mt][ks], acc[qr * 4 + mt][qc * 2 + nt]);
    __builtin_amdgcn_s_setprio(0);
  };
  auto wrap = [](int x) { return x >= RING_SLOTS ? x - RING_SLOTS : x; };
  using Q0 = std::integral_constant<int, 0>;
  using Q1 = std::integral_constant<int, 1>;

  // One phase P = 4t + j: reads, issue of half-tile P + D (when it exists; its kind
  // (j + D) & 3 is a compile-time constant), counted wait, barrier, MFMAs, barrier.
  // VM >= 0: that constant wait; VM == -2: the run-time wait of wait_at(P) (tail steps).
  auto wait_at = [&](int P) {  // what phase P+1 reads: half-tile P+2 (quadrants 0-2)
    if (P >= S - 1 || ((P + 1) & 3) == 3) return -1;
    const int last = P + D < S - 1 ? P + D : S - 1;
    return 2 * (last - (P + 2));
  };
  auto phase = [&](auto J, auto VM, int t, int rb) {
    constexpr int j = decltype(J)::value;
    constexpr int vmc = decltype(VM)::value;
    const int P = 4 * t + j;
    if constexpr (j == 0) { read_a(rb); read_b(Q0{}, wrap(rb + 1)); }
    if constexpr (j == 1) read_b(std::integral_constant<int, KEEPB ? 1 : 0>{}, wrap(rb + 2));
    if constexpr (j == 2) read_a(wrap(rb + 3));
    if constexpr (j == 3 && !KEEPB) read_b(Q0{}, wrap(rb + 1));
    const int si = P + D;
    if (vmc >= 0 || si < S) issue((j + D) & 3, si >> 2, si % RING_SLOTS);
    if constexpr (vmc >= 0)
      vm_wait<vmc>();
    else
      vm_wait_rt(wait_at(P));
    raw_barrier();
    if constexpr (j == 0) mfmas(Q0{}, Q0{});
    if constexpr (j == 1) mfmas(Q0{}, Q1{});
    if constexpr (j == 2) mfmas(Q1{}, Q1{});
    if constexpr (j == 3) mfmas(Q1{}, Q0{});
    raw_barrier();
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  using VSTEADY = std::integral_constant<int, 2 * (D - 2)>;
  using VTAIL = std::integral_constant<int, -2>;

  // prologue: half-tiles 0..D-1 in flight, wait for 0 and 1 (A0, B0 of step 0)
#pragma unroll
  for (int s = 0; s < D; ++s) issue(s & 3, s >> 2, s);
  vm_wait<2 * (D - 2)>();
  raw_barrier();
  if (wr == 1) raw_barrier();  // stagger: waves 4-7 one barrier behind

  int rb = 0;  // slot of the current step's A0 half-tile = (4t) % 10
  int t = 0;
  // steady state: all four phases issue (4t + 3 + D <= S - 1), constant wait
  for (; 4 * t + 3 + D <= S - 1; ++t) {
    phase(I0{}, VSTEADY{}, t, rb);
    phase(I1{}, VSTEADY{}, t, rb);
    phase(I2{}, VSTEADY{}, t, rb);
    phase(I3{}, VSTEADY{}, t, rb);
    rb = wrap(rb + 4);
  }
  // tail: the last (D + 3) / 4 steps issue what is left and drain with exact counts
  for (; t < nK; ++t) {
    phase(I0{}, VTAIL{}, t, rb);
    phase(I1{}, VTAIL{}, t, rb);
    phase(I2{}, VTAIL{}, t, rb);
    phase(I3{}, VTAIL{}, t, rb);
    rb = wrap(rb + 4);
  }
  if (wr == 0) raw_barrier();  // close the stagger

  if (nsl > 1) {  // ---- tail split: publish or combine
    __syncthreads();  // every wave is past its last LDS read: lds is free
    unsigned* ticket_lds = (unsigned*)lds;
    unsigned* cnt = st.cnt + sidx;
    unsigned* done = st.cnt + 8 * (st.tiles_per_xcd - st.full_per_xcd) + sidx;
    if (threadIdx.x == 0) ticket_lds[0] = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const unsigned ticket = ticket_lds[0];
    float* part = st.ws + (size_t)sidx * nsl * 65536;
    if (ticket + 1 < (unsigned)nsl) {  // not last: publish this slice's partial write-through
      unsigned long long* dst = (unsigned long long*)(part + (size_t)slice * 65536);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int hh = 0; hh < 2; ++hh) {
            const unsigned long long v = ((unsigned long long)__float_as_uint(acc[i][j][2 * hh + 1]) << 32) |
                                         __float_as_uint(acc[i][j][2 * hh]);
            __hip_atomic_store(dst + (((i * 4 + j) * 2 + hh) * 512 + threadIdx.x), v, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
          }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    // sc1 poll, then sc1 loads of the partials: no acquire fence (MI355X_MICROARCH.md,
    // visibility "Valid forms" row 1: one workgroup per CU, drained sc1 stores, one add per
    // storing workgroup behind its barrier; the other waves load after a barrier)
    if (threadIdx.x == 0) {
      while (__hip_atomic_load(done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1 < (unsigned)nsl)
        __builtin_amdgcn_s_sleep(2);
      __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    // fixed slice order, in place (a second 128-register accumulator would spill)
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          float v0 = 0.f, v1 = 0.f;
          for (int sl = 0; sl < nsl; ++sl) {
            if (sl == slice) {
              v0 += acc[i][j][2 * hh];
              v1 += acc[i][j][2 * hh + 1];
            } else {
              const unsigned long long* src = (const unsigned long long*)(part + (size_t)sl * 65536);
              const unsigned long long v = __hip_atomic_load(src + ((i * 4 + j) * 2 + hh) * 512 + threadIdx.x,
                                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              v0 += __uint_as_float((unsigned)v);
              v1 += __uint_as_float((unsigned)(v >> 32));
            }
          }
          acc[i][j][2 * hh] = v0;
          acc[i][j][2 * hh + 1] = v1;
        }
  }

  // ---- epilogue: lane holds C[row = ... + (lane & 15)][col = ... + 4 * (lane >> 4) + r]
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = m0 + wr * 128 + (i >> 2) * 64 + (i & 3) * 16 + (lane & 15);
    if (row >= M) continue;
    const float sc = rs ? rs[row] : 1.0f;  // folded RMSNorm row scale
    if constexpr (EPI == EPI_SILU) {
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const int col = n0 + wc * 32 + nt * 16 + 4 * (lane >> 4);
        u16x4 v;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float gg = rbf(acc[i][nt][r] * sc);
          const float uu = rbf(acc[i][2 + nt][r] * sc);
          v[r] = f2bf(rbf(silu_f(gg)) * uu);
        }
        *(u16x4*)(C + (int64_t)row * ldc + col) = v;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = n0 + wc * 64 + (j >> 1) * 32 + (j & 1) * 16 + 4 * (lane >> 4);
        u16x4 v;
        u16x4 rr;
        if constexpr (EPI == EPI_RESID) rr = *(const u16x4*)(R + (int64_t)row * ldr + col);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float o = acc[i][j][r] * sc;
          if constexpr (EPI == EPI_RESID) o = rbf(o) + bf2f(rr[r]);
          v[r] = f2bf(o);
        }
        *(u16x4*)(C + (int64_t)row * ldc + col) = v;
      }
    }
  }
}

// ============================================================ 4-wave 256x256 prefill GEMM
// gemm_w4_kernel: the same 256x256 output tile and K-step 64, on FOUR waves of 128x128
// (8x8 accumulator tiles = 256 AGPRs each, one wave per SIMD).  Per K-step a wave issues
// 128 MFMAs against 32 ds_read_b128 (0.25 LDS reads per MFMA; the 8-wave ring needs 0.375)
// and 3 barriers instead of 8, and its MFMA stream never waits for a partner wave.
//  * LDS: two K-step buffers of 64 KiB (A image [256 rows][128 B], XOR-swizzled 16-B
//    chunks; B image [16 n-tiles][2 k-halves][1 KiB] fragment-packed, lane-linear).
//  * Registers: F0 = the k-half-0 fragments (8 A + 8 B) of the current step, F1 = k-half 1.
//  * Iteration t (buffer c = t & 1): [A] MFMAs on F0 (rows 0-63) while F1 is read from c;
//    lgkmcnt(0) + barrier (every wave is done with c); [B] MFMAs on F0 (rows 64-127) and F1
//    (rows 0-63) while the 16 LDS-DMA pieces of step t+2 are issued into c; counted vmcnt
//    (step t+1's pieces landed) + barrier; [C] MFMAs on F1 (rows 64-127) while F0 of step
//    t+1 is read from c ^ 1.  Step t+1's pieces have one full iteration to land.
template <int EPI, int ORD>
__global__ __launch_bounds__(256, 1) void gemm_w4_kernel(
    const u16* __restrict__ A, int64_t lda, const u16* __restrict__ Wp, int KT, int n_tiles_w,
    u16* __restrict__ C, int64_t ldc, const u16* __restrict__ R, int64_t ldr, int M,
    const float* __restrict__ rs, int grid_m, int grid_n, SplitTail st) {
  __shared__ __attribute__((aligned(16))) char lds[2 * 65536];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wr = wave >> 1, wc = wave & 1;
  int bm, bn, slice = 0, nsl = 1, sidx = 0;
  tile_order(st, grid_m, grid_n, bm, bn, slice, nsl, sidx);
  const int m0 = bm * 256;
  const int n0 = bn * ((EPI == EPI_SILU) ? 128 : 256);
  const int nK = KT / 2 / nsl;  // 64-deep K-steps of this slice (>= 2)
  const int k0 = slice * nK;

  // ---- LDS-DMA sources: wave-uniform (SGPR) bases + per-lane 32-bit byte offsets, so
  // each piece is one global_load_lds with saddr: this wave's 8 A pieces (8 image rows
  // each) and 8 B pieces (one 1 KiB fragment tile each)
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  const char* a_base = (const char*)(A + (int64_t)m0 * lda + k0 * 64);
  unsigned a_voff[8];
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const int i = 64 * wave + 8 * p + (lane >> 3);  // image row 0..255
    const int rr = (m0 + i < M ? i : M - 1 - m0);
    const int chunk = (lane & 7) ^ ((i >> 1) & 7);
    a_voff[p] = (unsigned)(rr * lda * 2 + chunk * 16);
  }
  // B piece q = 8 * wave + p: image n-tile j = q >> 1, k-half q & 1
  int64_t b_soff[8];
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const int q = 8 * wv + p;
    const int j = q >> 1;
    int gnt;
    if constexpr (EPI == EPI_SILU) {  // wave column w: gate tiles 4w..4w+3, then the same up tiles
      const int w = j >> 3, jj = j & 7;
      gnt = (jj < 4 ? 0 : n_tiles_w / 2) + n0 / 16 + 4 * w + (jj & 3);
    } else {
      gnt = n0 / 16 + j;
    }
    b_soff[p] = ((int64_t)gnt * KT + 2 * k0 + (q & 1)) * 1024;
  }
  const unsigned b_voff = lane * 16;
  // ORD & 2: buffer_load_dwordx4 ... lds with the per-piece and per-step offsets in SGPRs
  // (soffset) instead of a 64-bit VGPR address per piece
  const __amdgpu_buffer_rsrc_t a_rsrc =
      __builtin_amdgcn_make_buffer_rsrc((void*)a_base, 0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t b_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)Wp, 0, 0x7fffffff, 0x00020000);
  auto issue = [&](int p, int t, int buf) {  // piece p (0-7 A, 8-15 B) of K-step t into buffer buf
    char* base = lds + buf * 65536;
    if constexpr ((ORD & 2) != 0) {
      typedef __attribute__((address_space(3))) void* lds_ptr;
      if (p < 8)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(a_rsrc, (lds_ptr)(base + (8 * wv + p) * 1024), 16, a_voff[p], t * 128,
                                                 0, 0);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(b_rsrc, (lds_ptr)(base + 32768 + (8 * wv + p - 8) * 1024), 16, b_voff,
                                                 (int)(b_soff[p - 8] + (int64_t)t * 2048), 0, 0);
    } else {
      if (p < 8)
        __builtin_amdgcn_global_load_lds((const void*)(a_base + t * 128 + a_voff[p]),
                                         (void*)(base + (8 * wv + p) * 1024), 16, 0, 0);
      else
        __builtin_amdgcn_global_load_lds((const void*)((const char*)Wp + b_soff[p - 8] + (int64_t)t * 2048 + b_voff),
                                         (void*)(base + 32768 + (8 * wv + p - 8) * 1024), 16, 0, 0);
    }
  };

  // ---- fragment reads: A rows wr*128 + mt*16 + (lane & 15), swizzle depends on lane only
  const int arow = wr * 128 + (lane & 15);
  const int a_off0 = arow * 128 + 16 * ((lane >> 4) ^ ((arow >> 1) & 7));
  const int a_off1 = arow * 128 + 16 * ((4 + (lane >> 4)) ^ ((arow >> 1) & 7));
  const int b_off = 32768 + (8 * wc) * 2048 + lane * 16;
  bf16x8 fa[2][8], fb[2][8];  // [k-half][tile]
  auto read_a = [&](int kh, int mt, int buf) {
    fa[kh][mt] = *(const bf16x8*)(lds + buf * 65536 + (kh ? a_off1 : a_off0) + mt * 2048);
  };
  auto read_b = [&](int kh, int nt, int buf) {
    fb[kh][nt] = *(const bf16x8*)(lds + buf * 65536 + b_off + nt * 2048 + kh * 1024);
  };
  // The 256 accumulators live in AGPRs through inline-asm MFMAs ("+a"): with the builtin,
  // hipcc's allocator rotates part of them through VGPRs inside the loop (copies per MFMA).
  // Hazards hipcc cannot see (cdna_hip_programming.md §5.7 item 2) are padded by hand:
  // zeroing -> first MFMA (acc_fence below), last MFMA -> first compiler read of a result.
  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto acc_fence = [&]() {  // 16 wait states, then every accumulator is redefined after them
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (i == 0)
        asm volatile("s_nop 7\n\ts_nop 7" : "+a"(acc[i][0]), "+a"(acc[i][1]), "+a"(acc[i][2]), "+a"(acc[i][3]),
                     "+a"(acc[i][4]), "+a"(acc[i][5]), "+a"(acc[i][6]), "+a"(acc[i][7]));
      else
        asm volatile("" : "+a"(acc[i][0]), "+a"(acc[i][1]), "+a"(acc[i][2]), "+a"(acc[i][3]), "+a"(acc[i][4]),
                     "+a"(acc[i][5]), "+a"(acc[i][6]), "+a"(acc[i][7]));
    }
  };
  acc_fence();
  auto mf = [&](int kh, int mt, int nt) {
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[mt][nt]) : "v"(fb[kh][nt]), "v"(fa[kh][mt]));
  };

  // MODE 0: steady (issue step t+2, wait for t+1, read F0 of t+1); 1: t = nK-2 (no issue,
  // wait 0, read); 2: t = nK-1 (no issue, no wait, no read)
  // MFMA x of a K-step (0..127) in issue order: [A] F0 rows 0-63, [B] F0 rows 64-127 then F1
  // rows 0-63, [C] F1 rows 64-127; ORD & 1 = nt-major inside each group of 32
  auto mfx = [&](int x) {
    const int kh = (x >= 64) ? 1 : 0;
    const int q = x & 31, half = (x >> 5) & 1;  // group of 32: rows 64 * half + ...
    if constexpr ((ORD & 1) == 0)
      mf(kh, 4 * half + (q >> 3), q & 7);
    else
      mf(kh, 4 * half + (q & 3), q >> 2);
  };
  // Every barrier is straddled by MFMAs (the last one before it is issued after the wait),
  // so the matrix pipe stays busy while the waves meet.
  auto iter = [&](auto MODE, int t) {
    constexpr int mode = decltype(MODE)::value;
    const int c = t & 1;
    // [A] 32 MFMAs; the 16 F1 reads from c ride the first 16
#pragma unroll
    for (int x = 0; x < 32; ++x) {
      if (x == 31) __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0), visible to hipcc's bookkeeping
      mfx(x);
      if (x < 16) {
        if (x < 8) read_b(1, x, c); else read_a(1, x - 8, c);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    raw_barrier();  // every wave is done reading c
    // [B] 64 MFMAs; the 16 LDS-DMA pieces of step t+2 into c, one after every 4th MFMA
#pragma unroll
    for (int x = 32; x < 96; ++x) {
      if (x == 95) {
        if constexpr (mode == 0) {
          vm_wait<16>();  // step t+1 landed (16 younger pieces in flight)
        } else if constexpr (mode == 1) {
          vm_wait<0>();
        }
      }
      mfx(x);
      if constexpr (mode == 0) {
        if ((x & 3) == 0) issue((x - 32) >> 2, t + 2, c);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    raw_barrier();  // step t+1 is visible in c ^ 1
    // [C] 32 MFMAs; F0 of step t+1 read from c ^ 1 during the first 16
#pragma unroll
    for (int x = 96; x < 128; ++x) {
      mfx(x);
      if constexpr (mode != 2) {
        if (x < 112) {
          if (x < 104) read_b(0, x - 96, c ^ 1); else read_a(0, x - 104, c ^ 1);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // prologue: steps 0 and 1 in flight, wait for step 0, read its F0
#pragma unroll
  for (int p = 0; p < 16; ++p) issue(p, 0, 0);
#pragma unroll
  for (int p = 0; p < 16; ++p) issue(p, 1, 1);
  vm_wait<16>();
  raw_barrier();
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    read_b(0, g, 0);
    read_a(0, g, 0);
  }
  int t = 0;
  for (; t < nK - 2; ++t) iter(std::integral_constant<int, 0>{}, t);
  iter(std::integral_constant<int, 1>{}, t);
  iter(std::integral_constant<int, 2>{}, t + 1);
  acc_fence();

  if (nsl > 1) {  // ---- tail split: publish or combine (as gemm_ring256_kernel)
    __syncthreads();
    unsigned* ticket_lds = (unsigned*)lds;
    unsigned* cnt = st.cnt + sidx;
    unsigned* done = st.cnt + 8 * (st.tiles_per_xcd - st.full_per_xcd) + sidx;
    if (threadIdx.x == 0) ticket_lds[0] = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const unsigned ticket = ticket_lds[0];
    float* part = st.ws + (size_t)sidx * nsl * 65536;
    if (ticket + 1 < (unsigned)nsl) {
      unsigned long long* dst = (unsigned long long*)(part + (size_t)slice * 65536);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
          for (int hh = 0; hh < 2; ++hh) {
            const unsigned long long v = ((unsigned long long)__float_as_uint(acc[i][j][2 * hh + 1]) << 32) |
                                         __float_as_uint(acc[i][j][2 * hh]);
            __hip_atomic_store(dst + (((i * 8 + j) * 2 + hh) * 256 + threadIdx.x), v, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
          }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    if (threadIdx.x == 0) {
      while (__hip_atomic_load(done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1 < (unsigned)nsl)
        __builtin_amdgcn_s_sleep(2);
      __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          float v0 = 0.f, v1 = 0.f;
          for (int sl = 0; sl < nsl; ++sl) {
            if (sl == slice) {
              v0 += acc[i][j][2 * hh];
              v1 += acc[i][j][2 * hh + 1];
            } else {
              const unsigned long long* src = (const unsigned long long*)(part + (size_t)sl * 65536);
              const unsigned long long v = __hip_atomic_load(src + ((i * 8 + j) * 2 + hh) * 256 + threadIdx.x,
                                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              v0 += __uint_as_float((unsigned)v);
              v1 += __uint_as_float((unsigned)(v >> 32));
            }
          }
          acc[i][j][2 * hh] = v0;
          acc[i][j][2 * hh + 1] = v1;
        }
  }

  // ---- epilogue: lane holds C[row = ... + (lane & 15)][col = ... + 4 * (lane >> 4) + r]
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = m0 + wr * 128 + i * 16 + (lane & 15);
    if (row >= M) continue;
    const float sc = rs ? rs[row] : 1.0f;
    if constexpr (EPI == EPI_SILU) {
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const int col = n0 + wc * 64 + nt * 16 + 4 * (lane >> 4);
        u16x4 v;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float gg = rbf(acc[i][nt][r] * sc);
          const float uu = rbf(acc[i][4 + nt][r] * sc);
          v[r] = f2bf(rbf(silu_f(gg)) * uu);
        }
        *(u16x4*)(C + (int64_t)row * ldc + col) = v;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int col = n0 + wc * 128 + j * 16 + 4 * (lane >> 4);
        u16x4 v;
        u16x4 rr;
        if constexpr (EPI == EPI_RESID) rr = *(const u16x4*)(R + (int64_t)row * ldr + col);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float o = acc[i][j][r] * sc;
          if constexpr (EPI == EPI_RESID) o = rbf(o) + bf2f(rr[r]);
          v[r] = f2bf(o);
        }
        *(u16x4*)(C + (int64_t)row * ldc + col) = v;
      }
    }
  }
}

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));


// EPI_QKV epilogue of one wave's 128 x 128 block = one head (q, k or v) of 128 rows: the
// arithmetic of qk_norm_rope_kv_kernel (elementwise.hip) on the accumulators.  Lane l holds
// rows row0 + 16 i + (l & 15), dims d = 16 nt + 4 (l >> 4) + r; the 4 lanes of a row (l,
// l^16, l^32, l^48) hold all 128 dims, and dims d and d + 64 (RoPE's rotate_half pair) sit
// in the same lane (nt and nt + 4).
__device__ __forceinline__ void qkv_epilogue(const f32x4 (&acc)[8][8], const QkvEpilogue& e, int row0, int hd, int M,
                                             const float* __restrict__ rs, int lane) {
  const int q4 = lane >> 4;  // dims 4*q4 .. 4*q4+3 of every 16-dim tile
  if (hd < e.H + e.KV) {
    const bool isq = hd < e.H;
    const u16* nw = isq ? e.qn_w : e.kn_w;
    u16x4 wv[8];
#pragma unroll
    for (int nt = 0; nt < 8; ++nt) wv[nt] = *(const u16x4*)(nw + 16 * nt + 4 * q4);
    // per-row operands up front, the cos/sin rows two-deep: the loads of row i+1 are in
    // flight while row i computes (dependent per-row loads were the epilogue's cost)
    int pos[8], slot[8];
    float scv[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = row0 + 16 * i + (lane & 15);
      const int rowc = row < M ? row : M - 1;
      pos[i] = e.positions[rowc];
      slot[i] = isq ? 0 : e.slots[rowc];
      scv[i] = rs ? rs[rowc] : 1.0f;
    }
    u16x4 cvb[2][4], svb[2][4];
    auto load_cs = [&](int i, int bsel) {
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        cvb[bsel][nt] = *(const u16x4*)(e.cos_t + (int64_t)pos[i] * 64 + 16 * nt + 4 * q4);
        svb[bsel][nt] = *(const u16x4*)(e.sin_t + (int64_t)pos[i] * 64 + 16 * nt + 4 * q4);
      }
    };
    load_cs(0, 0);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (i + 1 < 8) load_cs(i + 1, (i + 1) & 1);
      const int row = row0 + 16 * i + (lane & 15);
      const float sc = scv[i];
      float x[8][4];
      float ss = 0.f;
#pragma unroll
      for (int nt = 0; nt < 8; ++nt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          x[nt][r] = rbf(acc[i][nt][r] * sc);  // the bf16 projection output
          ss = fmaf(x[nt][r], x[nt][r], ss);
        }
      ss += __shfl_xor(ss, 16);
      ss += __shfl_xor(ss, 32);
      const float inv = 1.0f / sqrtf(ss / 128.0f + e.eps);
#pragma unroll
      for (int nt = 0; nt < 8; ++nt)
#pragma unroll
        for (int r = 0; r < 4; ++r) x[nt][r] = rbf(bf2f(wv[nt][r]) * rbf(x[nt][r] * inv));
      u16x4 o[8];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const u16x4 cv = cvb[i & 1][nt], sv = svb[i & 1][nt];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float c = bf2f(cv[r]), sn = bf2f(sv[r]);
          o[nt][r] = f2bf(rbf(x[nt][r] * c) + rbf(-x[nt + 4][r] * sn));
          o[nt + 4][r] = f2bf(rbf(x[nt + 4][r] * c) + rbf(x[nt][r] * sn));
        }
      }
      if (row >= M) continue;
      if (isq) {
        u16* qp = e.q_out + ((int64_t)row * e.H + hd) * HEAD_DIM + 4 * q4;
#pragma unroll
        for (int nt = 0; nt < 8; ++nt) *(u16x4*)(qp + 16 * nt) = o[nt];
      } else {
        if (slot[i] < 0) continue;
        const int page = slot[i] >> 6, s = slot[i] & 63, g = hd - e.H;
        u16* blk = e.kv_layer + kv_block(page, 0, g, e.KV);
#pragma unroll
        for (int nt = 0; nt < 8; ++nt) {  // K tile layout: 8-dim chunk c8 = d >> 3, element d & 7
          const int c8 = 2 * nt + (q4 >> 1);
          const int ln = (s & 15) + 16 * (c8 & 3);
          *(u16x4*)(blk + (((s >> 4) * 4 + (c8 >> 2)) * 64 + ln) * 8 + 4 * (q4 & 1)) = o[nt];
        }
      }
    }
  } else {  // v head: the bf16 projection output, scattered into the V^T tile layout
    const int g = hd - e.H - e.KV;
    int slots[8];
    float scv[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int rowc = min(row0 + 16 * i + (lane & 15), M - 1);
      slots[i] = e.slots[rowc];
      scv[i] = rs ? rs[rowc] : 1.0f;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = row0 + 16 * i + (lane & 15);
      if (row >= M) continue;
      const int slot = slots[i];
      if (slot < 0) continue;
      const float sc = scv[i];
      const int page = slot >> 6, s = slot & 63;
      u16* blk = e.kv_layer + kv_block(page, 1, g, e.KV);
      const int kt = s >> 5, tp = s & 31;
      const int gg = tp < 16 ? (tp >> 2) : ((tp - 16) >> 2);
      const int jj = tp < 16 ? (tp & 3) : 4 + ((tp - 16) & 3);
#pragma unroll
      for (int nt = 0; nt < 8; ++nt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int ln = 4 * q4 + r + 16 * gg;  // d & 15 = 4 q4 + r, d >> 4 = nt
          blk[((kt * 8 + nt) * 64 + ln) * 8 + jj] = f2bf(acc[i][nt][r] * sc);
        }
    }
  }
}

// ============================================================ persistent 4-wave GEMM
// gemm_w4p_kernel: gemm_w4_kernel's K-loop, but one workgroup per CU walks the units
// v = blockIdx.x, + gridDim.x, ... (gridDim.x a multiple of 8, so every unit keeps the XCD
// that tile_order gives it), and the next unit's K-steps 0 and 1 are issued into the LDS
// buffers as soon as the current unit's last two steps free them (phase B of its last two
// iterations), i.e. BEFORE the epilogue: the next tile's HBM latency overlaps the store
// tail instead of following it.  The first K-step of a unit starts its accumulators with a
// zero C operand (no zeroing pass).  Buffer of step t = (t + par) & 1, par carried across
// units.  Whole tiles only: grids that need the tail split run gemm_w4_kernel.
template <int EPI>
__global__ __launch_bounds__(256, 1) void gemm_w4p_kernel(
    const u16* __restrict__ A, int64_t lda, const u16* __restrict__ Wp, int KT, int n_tiles_w,
    u16* __restrict__ C, int64_t ldc, const u16* __restrict__ R, int64_t ldr, int M,
    const float* __restrict__ rs, int grid_m, int grid_n, SplitTail st, int nunits, QkvEpilogue qe) {
  __shared__ __attribute__((aligned(16))) char lds[2 * 65536 + 16];  // + the split ticket
  typedef __attribute__((address_space(3))) void* lds_ptr;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wr = wave >> 1, wc = wave & 1;
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  // vector-memory operations per wave in one epilogue (+8 row-scale loads when rs)
  constexpr int EPI_OPS = EPI == EPI_SILU ? 32 : EPI == EPI_RESID ? 128 : 64;
  const __amdgpu_buffer_rsrc_t c_rsrc =
      __builtin_amdgcn_make_buffer_rsrc((void*)C, 0, (int)((int64_t)M * ldc * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t r_rsrc =
      __builtin_amdgcn_make_buffer_rsrc((void*)R, 0, R ? (int)((int64_t)M * ldr * 2) : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)rs, 0, rs ? M * 4 : 0, 0x00020000);

  struct Unit {
    int m0, n0, nK, slice, nsl, sidx;
  };
  // LDS-DMA sources of the unit being loaded: buffer descriptors + per-piece offsets
  __amdgpu_buffer_rsrc_t src_a, src_b;
  unsigned a_voff[8];
  int b_soff[8];
  auto unit_of = [&](int v) {
    Unit u;
    int bm, bn;
    u.slice = 0;
    u.nsl = 1;
    u.sidx = 0;
    tile_order_v(st, grid_m, grid_n, v, nunits, bm, bn, u.slice, u.nsl, u.sidx);
    u.m0 = bm * 256;
    u.n0 = bn * ((EPI == EPI_SILU) ? 128 : 256);
    u.nK = KT / 2 / u.nsl;
    return u;
  };
  auto gnt_of = [&](const Unit& u, int p) {  // B piece q = 8 * wave + p: n-tile j = q >> 1, k-half q & 1
    const int j = (8 * wv + p) >> 1;
    if constexpr (EPI == EPI_SILU) {  // wave column w: gate tiles 4w..4w+3, then the same up tiles
      const int w = j >> 3, jj = j & 7;
      return (jj < 4 ? 0 : n_tiles_w / 2) + u.n0 / 16 + 4 * w + (jj & 3);
    } else {
      return u.n0 / 16 + j;
    }
  };
  auto src_of = [&](const Unit& u) {
    const int k0 = u.slice * u.nK;
    src_a = __builtin_amdgcn_make_buffer_rsrc((void*)(A + (int64_t)u.m0 * lda + k0 * 64), 0, 0x7fffffff, 0x00020000);
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      const int i = 64 * wave + 8 * p + (lane >> 3);  // image row 0..255
      const int rr = (u.m0 + i < M ? i : M - 1 - u.m0);
      const int chunk = (lane & 7) ^ ((i >> 1) & 7);
      a_voff[p] = (unsigned)(rr * lda * 2 + chunk * 16);
    }
    const int g0 = gnt_of(u, 0);
    src_b = __builtin_amdgcn_make_buffer_rsrc((void*)(Wp + ((int64_t)g0 * KT + 2 * k0) * 512), 0, 0x7fffffff,
                                             0x00020000);
#pragma unroll
    for (int p = 0; p < 8; ++p) b_soff[p] = ((gnt_of(u, p) - g0) * KT + (p & 1)) * 1024;
  };
  auto issue = [&](int p, int t, int buf) {  // piece p (0-7 A, 8-15 B) of K-step t
    char* base = lds + buf * 65536;
    if (p < 8)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(src_a, (lds_ptr)(base + (8 * wv + p) * 1024), 16, a_voff[p],
                                               t * 128, 0, 0);
    else
      __builtin_amdgcn_raw_ptr_buffer_load_lds(src_b, (lds_ptr)(base + 32768 + (8 * wv + p - 8) * 1024), 16,
                                               lane * 16, b_soff[p - 8] + t * 2048, 0, 0);
  };

  const int arow = wr * 128 + (lane & 15);
  const int a_off0 = arow * 128 + 16 * ((lane >> 4) ^ ((arow >> 1) & 7));
  const int a_off1 = arow * 128 + 16 * ((4 + (lane >> 4)) ^ ((arow >> 1) & 7));
  const int b_off = 32768 + (8 * wc) * 2048 + lane * 16;
  bf16x8 fa[2][8], fb[2][8];  // [k-half][tile]
  auto read_a = [&](int kh, int mt, int buf) {
    fa[kh][mt] = *(const bf16x8*)(lds + buf * 65536 + (kh ? a_off1 : a_off0) + mt * 2048);
  };
  auto read_b = [&](int kh, int nt, int buf) {
    fb[kh][nt] = *(const bf16x8*)(lds + buf * 65536 + b_off + nt * 2048 + kh * 1024);
  };
  f32x4 acc[8][8];
  auto acc_fence = [&]() {  // 16 wait states after the last MFMA, then every accumulator redefined
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (i == 0)
        asm volatile("s_nop 7\n\ts_nop 7" : "+a"(acc[i][0]), "+a"(acc[i][1]), "+a"(acc[i][2]), "+a"(acc[i][3]),
                     "+a"(acc[i][4]), "+a"(acc[i][5]), "+a"(acc[i][6]), "+a"(acc[i][7]));
      else
        asm volatile("" : "+a"(acc[i][0]), "+a"(acc[i][1]), "+a"(acc[i][2]), "+a"(acc[i][3]), "+a"(acc[i][4]),
                     "+a"(acc[i][5]), "+a"(acc[i][6]), "+a"(acc[i][7]));
    }
  };
  // MFMA x of a K-step (0..127), nt-major inside each group of 32 (see gemm_w4_kernel);
  // ZERO: the unit's first K-step, k-half 0 starts the accumulator from 0
  auto mfx = [&](bool zero, int x) {  // zero: compile-time after inlining
    const int kh = (x >= 64) ? 1 : 0;
    const int q = x & 31, half = (x >> 5) & 1;
    const int mt = 4 * half + (q & 3), nt = q >> 2;
    if (zero && kh == 0)
      asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(acc[mt][nt]) : "v"(fb[0][nt]), "v"(fa[0][mt]));
    else
      asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[mt][nt]) : "v"(fb[kh][nt]), "v"(fa[kh][mt]));
  };
  using ZF = std::integral_constant<bool, false>;
  using ZT = std::integral_constant<bool, true>;
  // MODE 0: issue step t+2, wait for t+1, read F0 of t+1; 1 (t = nK-2): issue the next
  // unit's step 0 (if any), wait for t+1, read; 2 (t = nK-1): issue the next unit's step 1
  auto iter = [&](auto MODE, auto ZERO, int t, int par, bool has_next) {
    constexpr int mode = decltype(MODE)::value;
    const int c = (t + par) & 1;
#pragma unroll
    for (int x = 0; x < 32; ++x) {
      if (x == 31) __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
      mfx(decltype(ZERO)::value, x);
      if (x < 16) {
        if (x < 8) read_b(1, x, c); else read_a(1, x - 8, c);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    raw_barrier();  // every wave is done reading buffer c
#pragma unroll
    for (int x = 32; x < 96; ++x) {
      if (x == 95) {
        if constexpr (mode == 0) {
          vm_wait<16>();
        } else if constexpr (mode == 1) {
          if (has_next) vm_wait<16>(); else vm_wait<0>();
        }
      }
      mfx(decltype(ZERO)::value, x);
      if ((x & 3) == 0) {
        if constexpr (mode == 0) {
          issue((x - 32) >> 2, t + 2, c);
        } else {
          if (has_next) issue((x - 32) >> 2, mode == 1 ? 0 : 1, c);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    raw_barrier();  // step t+1 visible in buffer c ^ 1
#pragma unroll
    for (int x = 96; x < 128; ++x) {
      mfx(decltype(ZERO)::value, x);
      if constexpr (mode != 2) {
        if (x < 112) {
          if (x < 104) read_b(0, x - 96, c ^ 1); else read_a(0, x - 104, c ^ 1);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  int v = blockIdx.x;
  Unit u = unit_of(v);
  src_of(u);
  int par = 0;
#pragma unroll
  for (int p = 0; p < 16; ++p) issue(p, 0, 0);
#pragma unroll
  for (int p = 0; p < 16; ++p) issue(p, 1, 1);
  bool first = true;
  for (;;) {
    // step 0 landed: younger than its pieces are step 1's 16 and, after the first unit, the
    // previous epilogue's EPI_OPS (fewer only when a split slice drained with vmcnt(0))
    if (first || EPI == EPI_QKV) {  // EPI_QKV: its epilogue's count varies by head kind
      vm_wait<16>();
    } else if (rs) {
      vm_wait<(16 + EPI_OPS + 8 < 63 ? 16 + EPI_OPS + 8 : 63)>();
    } else {
      vm_wait<(16 + EPI_OPS < 63 ? 16 + EPI_OPS : 63)>();
    }
    first = false;
    raw_barrier();
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      read_b(0, g, par);
      read_a(0, g, par);
    }
    iter(std::integral_constant<int, 0>{}, ZT{}, 0, par, false);
    for (int t = 1; t < u.nK - 2; ++t) iter(std::integral_constant<int, 0>{}, ZF{}, t, par, false);
    // this unit's loads are all issued: cur now describes the next unit
    const int vn = v + gridDim.x;
    const bool has_next = vn < nunits;
    Unit un = u;
    // EPI_QKV: no cross-tile prefetch -- its epilogue's own loads (positions, cos/sin,
    // slots) would wait behind the next tile's 32 in-flight pieces (in-order vmcnt); the
    // next tile's sources are then computed after the epilogue (fewer live registers in it)
    constexpr bool XPF = EPI != EPI_QKV;
    if (has_next) {
      un = unit_of(vn);
      if constexpr (XPF) src_of(un);
    }
    iter(std::integral_constant<int, 1>{}, ZF{}, u.nK - 2, par, XPF && has_next);
    iter(std::integral_constant<int, 2>{}, ZF{}, u.nK - 1, par, XPF && has_next);
    acc_fence();

    if constexpr (EPI == EPI_QKV) {
      qkv_epilogue(acc, qe, u.m0 + wr * 128, (u.n0 >> 7) + wc, M, rs, lane);
    } else {  // ---- epilogue: lane holds C[row = ... + (lane & 15)][col = ... + 4 * (lane >> 4) + r]
      // buffer loads/stores: rows >= M are issued and dropped by the range check, so the
      // epilogue's vector-memory count is fixed (EPI_OPS) and the next unit's wait is exact
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int row = u.m0 + wr * 128 + i * 16 + (lane & 15);
        float sc = 1.0f;
        if (rs) sc = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs_rsrc, row * 4, 0, 0));
        if constexpr (EPI == EPI_SILU) {
#pragma unroll
          for (int nt = 0; nt < 4; ++nt) {
            const int col = u.n0 + wc * 64 + nt * 16 + 4 * (lane >> 4);
            u16x4 o;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float gg = rbf(acc[i][nt][r] * sc);
              const float uu = rbf(acc[i][4 + nt][r] * sc);
              o[r] = f2bf(rbf(silu_f(gg)) * uu);
            }
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, o), c_rsrc, (row * (int)ldc + col) * 2, 0,
                                                  0);
          }
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int col = u.n0 + wc * 128 + j * 16 + 4 * (lane >> 4);
            u16x4 o;
            u16x4 rr;
            if constexpr (EPI == EPI_RESID)
              rr = __builtin_bit_cast(u16x4, __builtin_amdgcn_raw_buffer_load_b64(r_rsrc, (row * (int)ldr + col) * 2,
                                                                                   0, 0));
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              float x = acc[i][j][r] * sc;
              if constexpr (EPI == EPI_RESID) x = rbf(x) + bf2f(rr[r]);
              o[r] = f2bf(x);
            }
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, o), c_rsrc, (row * (int)ldc + col) * 2, 0,
                                                  0);
          }
        }
      }
    }
    if (!has_next) break;
    par = (par + u.nK) & 1;
    u = un;
    v = vn;
    if constexpr (!XPF) {  // the next tile's steps 0 and 1, issued after the epilogue
      src_of(u);
#pragma unroll
      for (int p = 0; p < 16; ++p) issue(p, 0, par);
#pragma unroll
      for (int p = 0; p < 16; ++p) issue(p, 1, par ^ 1);
    }
  }
}

// INFERD_GEMM_TILE selects the prefill GEMM (read per call so one process can A/B them):
// "w4p" (default: persistent w4, w4 where the grid needs a tail split) | "w4" ("w4m" / "w4g" /
// "w4mg" its A/B arms) | "ring" | "256" | "128"
static int gemm_tile_variant() {
  const char* e = getenv("INFERD_GEMM_TILE");
  if (!e || !*e) return 8;
  if (e[0] == 'r') return 0;
  if (e[0] == 'w' && e[2] == 'p') return 8;  // "w4p": persistent
  if (e[0] == 'w') {  // "w4" = "w4nb" (default) | "w4m": mt-major MFMA order | "w4g": global_load_lds
    int v = 7;
    for (const char* c = e + 2; *c; ++c) v &= (*c == 'm') ? ~1 : (*c == 'g') ? ~2 : ~0;
    return v;
  }
  return atoi(e);
}

// Tail-split plan for `tiles` 256x256 tiles of nK K-steps on 8 XCDs x 32 CUs (one 512-thread
// workgroup per CU).  INFERD_GEMM_SPLIT=0 disables it.  The fp32 partial workspace and the
// counters are allocated once (zeroed) and grown on demand; never inside a graph capture.
static int env_or(const char* name, int dflt) {
  const char* e = getenv(name);
  return e && *e ? atoi(e) : dflt;
}

template <int EPI>
static void ring_launch(bool keepb, int grid, hipStream_t s, const u16* A, int64_t lda, const u16* Wp, int KT, int ntw,
                        u16* C, int64_t ldc, const u16* R, int64_t ldr, int M, const float* rs, int gm, int gn,
                        const SplitTail& st) {
  if (keepb)
    hipLaunchKernelGGL((gemm_ring256_kernel<EPI, true>), dim3(grid), dim3(512), 0, s, A, lda, Wp, KT, ntw, C, ldc, R,
                       ldr, M, rs, gm, gn, st);
  else
    hipLaunchKernelGGL((gemm_ring256_kernel<EPI, false>), dim3(grid), dim3(512), 0, s, A, lda, Wp, KT, ntw, C, ldc, R,
                       ldr, M, rs, gm, gn, st);
}

#define SPLIT_MAX_DEVICES_ 16
template <int ORD>
static void w4_launch(int epi, int grid, hipStream_t s, const u16* A, int64_t lda, const u16* Wp, int KT, int ntw,
                      u16* C, int64_t ldc, const u16* R, int64_t ldr, int M, const float* rs, int gm, int gn,
                      const SplitTail& st) {
  switch (epi) {
    case EPI_NONE:
      hipLaunchKernelGGL((gemm_w4_kernel<EPI_NONE, ORD>), dim3(grid), dim3(256), 0, s, A, lda, Wp, KT, ntw, C, ldc, R,
                         ldr, M, rs, gm, gn, st);
      break;
    case EPI_RESID:
      hipLaunchKernelGGL((gemm_w4_kernel<EPI_RESID, ORD>), dim3(grid), dim3(256), 0, s, A, lda, Wp, KT, ntw, C, ldc,
                         R, ldr, M, rs, gm, gn, st);
      break;
    default:
      hipLaunchKernelGGL((gemm_w4_kernel<EPI_SILU, ORD>), dim3(grid), dim3(256), 0, s, A, lda, Wp, KT, ntw, C, ldc,
                         R, ldr, M, rs, gm, gn, st);
      break;
  }
}

// persistent grid: one workgroup per CU, a multiple of 8 (units keep their XCD), <= units
static int w4p_grid(int units) {
  static int ncu[SPLIT_MAX_DEVICES_] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= SPLIT_MAX_DEVICES_) dev = 0;
  if (ncu[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    ncu[dev] = n;
  }
  const int cap = env_or("INFERD_W4P_GRID", 0) > 0 ? env_or("INFERD_W4P_GRID", 0) : ncu[dev];
  if (units <= cap) return units;
  return cap & ~7;
}

// Per device (a process may drive several GPUs); grown on demand, never inside a graph
// capture, not thread-safe (one host thread per device, like the span API).
#define SPLIT_MAX_DEVICES 16
struct SplitWs {
  float* ws = nullptr;
  size_t ws_bytes = 0;
  unsigned* cnt = nullptr;
  int cnt_n = 0;
};
static SplitWs g_split[SPLIT_MAX_DEVICES];

static SplitTail plan_split_tail(int tiles, int nK, hipStream_t s) {
  SplitTail st = {1, 0, 0, 0, nullptr, nullptr};
  const char* e = getenv("INFERD_GEMM_SPLIT");
  if (e && *e && atoi(e) == 0) return st;
  if (tiles % 8) return st;
  const int per = tiles / 8, rem = per % 32;
  if (rem == 0 || 32 % rem) return st;
  const int split = 32 / rem;
  if (split > 8 || nK % split || nK / split < 3) return st;
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cap) != hipSuccess || cap != hipStreamCaptureStatusNone) return st;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= SPLIT_MAX_DEVICES) return st;
  SplitWs& w = g_split[dev];
  const size_t bytes = (size_t)8 * rem * split * 65536 * sizeof(float);
  if (bytes > w.ws_bytes) {
    if (w.ws) (void)hipFree(w.ws);
    w.ws = nullptr;
    w.ws_bytes = 0;
    if (hipMalloc((void**)&w.ws, bytes) != hipSuccess) return st;
    w.ws_bytes = bytes;
  }
  if (2 * 8 * rem > w.cnt_n) {
    if (w.cnt) (void)hipFree(w.cnt);
    w.cnt = nullptr;
    w.cnt_n = 0;
    if (hipMalloc((void**)&w.cnt, 2 * 8 * rem * sizeof(unsigned)) != hipSuccess) return st;
    if (hipMemset(w.cnt, 0, 2 * 8 * rem * sizeof(unsigned)) != hipSuccess) return st;
    w.cnt_n = 2 * 8 * rem;
  }
  st.split = split;
  st.tiles_per_xcd = per;
  st.full_per_xcd = per - rem;
  st.units_per_xcd = per - rem + rem * split;
  st.ws = w.ws;
  st.cnt = w.cnt;
  return st;
}

static bool use_ring256(int M, int N, int K, int epi) {
  const int v = gemm_tile_variant();
  if ((v != 0 && (v < 4 || v > 8)) || M < 512 || K < 192) return false;
  return (epi == EPI_SILU) ? (N % 128 == 0) : (N % 256 == 0);
}

static bool use_tiled256(int M, int N, int epi) {
  if (gemm_tile_variant() == 128 || M < 512) return false;
  return (epi == EPI_SILU) ? (N % 128 == 0) : (N % 256 == 0);
}

// ============================================================ dispatch
bool gemm_uses_tiled(int M, int N, int K, int epi) {
  return (M > 64) && (K % TBK == 0) && ((epi == EPI_SILU) ? (N % 64 == 0) : (N % TBN == 0)) &&
         epi != EPI_ARGMAX;
}

void launch_gemm(const u16* A, int64_t lda, const u16* Wp, int M, int N, int K, u16* C, int64_t ldc,
                 const u16* R, int64_t ldr, int epi, unsigned long long* keys, hipStream_t s,
                 const RowNorm* norm) {
  const int KT = K / 32;
  const int n_tiles = N / 16;  // output tiles of 16 columns
  const float* rs = nullptr;
  if (norm && gemm_uses_tiled(M, N, K, epi)) {
    launch_row_inv_rms(A, lda, M, K, norm->eps, norm->rs_ws, s);
    rs = norm->rs_ws;
  }
  if (gemm_uses_tiled(M, N, K, epi) && use_ring256(M, N, K, epi)) {
    const int ncols = (epi == EPI_SILU) ? 128 : 256;
    const int gm = (M + 255) / 256, gn = N / ncols;
    const int ntw = (epi == EPI_SILU) ? 2 * n_tiles : n_tiles;
    const SplitTail st = plan_split_tail(gm * gn, K / 64, s);
    const int grid = st.split > 1 ? 8 * st.units_per_xcd : gm * gn;
    // INFERD_GEMM_KEEPB=0 selects the look-ahead-6 schedule that re-reads B0 (A/B)
    const bool keepb = env_or("INFERD_GEMM_KEEPB", 1) != 0;
    // w4p addresses C / R through 32-bit buffer offsets
    const bool fits32 = (int64_t)(M + 256) * ldc * 2 < 0x7fffffff && (!R || (int64_t)(M + 256) * ldr * 2 < 0x7fffffff);
    if (gemm_tile_variant() == 8 && fits32 && st.split == 1) {
      const int g = w4p_grid(grid);
      switch (epi) {
        case EPI_NONE:
          hipLaunchKernelGGL(gemm_w4p_kernel<EPI_NONE>, dim3(g), dim3(256), 0, s, A, lda, Wp, KT, ntw, C, ldc, R, ldr,
                             M, rs, gm, gn, st, grid, QkvEpilogue{});
          break;
        case EPI_RESID:
          hipLaunchKernelGGL(gemm_w4p_kernel<EPI_RESID>, dim3(g), dim3(256), 0, s, A, lda, Wp, KT, ntw, C, ldc, R, ldr,
                             M, rs, gm, gn, st, grid, QkvEpilogue{});
          break;
        default:
          hipLaunchKernelGGL(gemm_w4p_kernel<EPI_SILU>, dim3(g), dim3(256), 0, s, A, lda, Wp, KT, ntw, C, ldc, R, ldr,
                             M, rs, gm, gn, st, grid, QkvEpilogue{});
          break;
      }
      return;
    }
    if (gemm_tile_variant() >= 4 && gemm_tile_variant() <= 8) {  // w4p with a tail split: w4
      switch (gemm_tile_variant()) {
        case 4: w4_launch<0>(epi, grid, s, A, lda, Wp, KT, ntw, C, ldc, R, ldr, M, rs, gm, gn, st); break;
        case 5: w4_launch<1>(epi, grid, s, A, lda, Wp, KT, ntw, C, ldc, R, ldr, M, rs, gm, gn, st); break;
        case 6: w4_launch<2>(epi, grid, s, A, lda, Wp, KT, ntw, C, ldc, R, ldr, M, rs, gm, gn, st); break;
        default: w4_launch<3>(epi, grid, s, A, lda, Wp, KT, ntw, C, ldc, R, ldr, M, rs, gm, gn, st); break;
      }
      return;
    }
    switch (epi) {
      case EPI_NONE:
        ring_launch<EPI_NONE>(keepb, grid, s, A, lda, Wp, KT, ntw, C, ldc, R, ldr, M, rs, gm, gn, st);
        break;
      case EPI_RESID:
        ring_launch<EPI_RESID>(keepb, grid, s, A, lda, Wp, KT, ntw, C, ldc, R, ldr, M, rs, gm, gn, st);
        break;
      default:
        ring_launch<EPI_SILU>(keepb, grid, s, A, lda, Wp, KT, ntw, C, ldc, R, ldr, M, rs, gm, gn, st);
        break;
    }
    return;
  }
  if (gemm_uses_tiled(M, N, K, epi) && use_tiled256(M, N, epi)) {
    const int ncols = (epi == EPI_SILU) ? 128 : 256;
    dim3 g(N / ncols, (M + 255) / 256);
    const int ntw = (epi == EPI_SILU) ? 2 * n_tiles : n_tiles;
    switch (epi) {
      case EPI_NONE:
        hipLaunchKernelGGL(gemm_tiled256_kernel<EPI_NONE>, g, dim3(512), 0, s, A, lda, Wp, KT, ntw, C, ldc, R, ldr, M, rs);
        break;
      case EPI_RESID:
        hipLaunchKernelGGL(gemm_tiled256_kernel<EPI_RESID>, g, dim3(512), 0, s, A, lda, Wp, KT, ntw, C, ldc, R, ldr, M, rs);
        break;
      default:
        hipLaunchKernelGGL(gemm_tiled256_kernel<EPI_SILU>, g, dim3(512), 0, s, A, lda, Wp, KT, ntw, C, ldc, R, ldr, M, rs);
        break;
    }
    return;
  }
  if (gemm_uses_tiled(M, N, K, epi)) {
    const int ncols = (epi == EPI_SILU) ? 64 : 128;
    dim3 g(N / ncols, (M + TBM - 1) / TBM);
    const int ntw = (epi == EPI_SILU) ? 2 * n_tiles : n_tiles;
    switch (epi) {
      case EPI_NONE:
        hipLaunchKernelGGL(gemm_tiled_kernel<EPI_NONE>, g, dim3(256), 0, s, A, lda, Wp, KT, ntw, C, ldc, R, ldr, M, rs);
        break;
      case EPI_RESID:
        hipLaunchKernelGGL(gemm_tiled_kernel<EPI_RESID>, g, dim3(256), 0, s, A, lda, Wp, KT, ntw, C, ldc, R, ldr, M, rs);
        break;
      default:
        hipLaunchKernelGGL(gemm_tiled_kernel<EPI_SILU>, g, dim3(256), 0, s, A, lda, Wp, KT, ntw, C, ldc, R, ldr, M, rs);
        break;
    }
    return;
  }
  // decode path, 64-row slabs (M > 64 only when the tiled shape constraints fail)
  for (int m0 = 0; m0 < M; m0 += 64) {
    DecodeArgs a = {};
    a.M = (M - m0) < 64 ? (M - m0) : 64;
    a.A = A + (int64_t)m0 * lda;
    a.lda = lda;
    a.Wp = Wp;
    a.KT = KT;
    a.n_tiles = n_tiles;
    a.C = C ? C + (int64_t)m0 * ldc : nullptr;
    a.ldc = ldc;
    a.R = R ? R + (int64_t)m0 * ldr : nullptr;
    a.ldr = ldr;
    a.keys = keys;
    a.eps = norm ? norm->eps : 0.f;
    if (norm) {
      switch (epi) {
        case EPI_NONE: decode_mt<EPI_NONE, true>(a, s); break;
        case EPI_SILU: decode_mt<EPI_SILU, true>(a, s); break;
        default: return;  // the span folds norms into the NONE (qkv) and SILU (gate/up) GEMMs only
      }
    } else {
      switch (epi) {
        case EPI_NONE: decode_mt<EPI_NONE, false>(a, s); break;
        case EPI_RESID: decode_mt<EPI_RESID, false>(a, s); break;
        case EPI_SILU: decode_mt<EPI_SILU, false>(a, s); break;
        default: decode_mt<EPI_ARGMAX, false>(a, s); break;
      }
    }
    if (epi == EPI_ARGMAX) break;  // argmax requires M <= 64 (checked by the caller)
  }
}

// Greedy id per row from the lm_head GEMV's per-tile keys (layout [M][n_tiles], so a
// row's keys are contiguous): one 1024-thread workgroup per row, four independent
// coalesced loads in flight per thread, max over (value key << 32 | ~col) = the first
// maximal column, as torch.argmax.
__global__ __launch_bounds__(1024) void argmax_reduce_kernel(const unsigned long long* __restrict__ partial,
                                                             int n_tiles, int32_t* __restrict__ ids) {
  __shared__ unsigned long long red[16];
  const int row = blockIdx.x;
  const unsigned long long* p = partial + (int64_t)row * n_tiles;
  unsigned long long best = 0;
  for (int t = threadIdx.x; t < n_tiles; t += 4 * 1024) {
    unsigned long long k[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) k[u] = (t + u * 1024 < n_tiles) ? p[t + u * 1024] : 0ull;
#pragma unroll
    for (int u = 0; u < 4; ++u) best = k[u] > best ? k[u] : best;
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
    for (int w = 1; w < 16; ++w) b = red[w] > b ? red[w] : b;
    ids[row] = (int32_t)(0xFFFFFFFFu - (uint32_t)(b & 0xFFFFFFFFull));
  }
}

void launch_argmax_reduce(const unsigned long long* partial, int n_tiles, int M, int32_t* ids,
                          hipStream_t s) {
  hipLaunchKernelGGL(argmax_reduce_kernel, dim3(M), dim3(1024), 0, s, partial, n_tiles, ids);
}

// ============================================================ fused prefill q/k/v projection
// launch_gemm's persistent whole-tile path with the EPI_QKV epilogue: q/k RMSNorm + RoPE to
// q_out and the K cache, V to the cache (what launch_qk_norm_rope_kv does from a stored q/k/v
// row).  Needs that path: the 4-wave persistent kernel selected, no tail split, 32-bit C offsets
// (C is unused here) and one head per wave column (N = (H + 2 KV) * 128).
// INFERD_FUSE_QKV_EPI=0 keeps the two-kernel path (A/B).
bool launch_gemm_qkv_fused(const u16* A, int64_t lda, const u16* Wp, int M, int N, int K, const RowNorm* norm,
                           const QkvEpilogue& e, hipStream_t s) {
  if (env_or("INFERD_FUSE_QKV_EPI", 1) == 0) return false;
  if (gemm_tile_variant() != 8 || !gemm_uses_tiled(M, N, K, EPI_NONE) || !use_ring256(M, N, K, EPI_NONE)) return false;
  if (N != (e.H + 2 * e.KV) * HEAD_DIM) return false;
  const int gm = (M + 255) / 256, gn = N / 256;
  const int tiles = gm * gn, nK = K / 64;
  // the tail-split decision of plan_split_tail, without its workspace
  if (tiles % 8 == 0) {
    const int rem = (tiles / 8) % 32;
    if (rem != 0 && 32 % rem == 0) {
      const int split = 32 / rem;
      if (split <= 8 && nK % split == 0 && nK / split >= 3) return false;
    }
  }
  const float* rs = nullptr;
  if (norm) {
    launch_row_inv_rms(A, lda, M, K, norm->eps, norm->rs_ws, s);
    rs = norm->rs_ws;
  }
  const SplitTail st = {1, 0, 0, 0, nullptr, nullptr};
  hipLaunchKernelGGL(gemm_w4p_kernel<EPI_QKV>, dim3(w4p_grid(tiles)), dim3(256), 0, s, A, lda, Wp, K / 32, N / 16,
                     (u16*)nullptr, (int64_t)0, (const u16*)nullptr, (int64_t)0, M, rs, gm, gn, st, tiles, e);
  return true;
}
