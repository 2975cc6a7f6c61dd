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
//  * gemm_w4p / gemm_w4: >= 512 rows (prefill).  256x256x64 block tiles on four waves,
//    LDS-DMA staged (see their section); gemm_tiled: 65..511 rows and odd shapes, 128x128
//    tiles, double-buffered LDS with global_load_lds (A XOR-swizzled on the source address,
//    B already fragment-ordered).
#include <stdlib.h>

#include <utility>

#include "common.h"
#include "kernels.h"

// SiLU of the bf16 gate value g in fp32 (torch: x / (1 + exp(-x)) in float opmath, then bf16):
// v_exp_f32 on -g * log2 e and v_rcp_f32 instead of the libm expf and an IEEE division (~18
// VALU -> 4 per element in the prefill gate/up epilogue, which runs exposed between tiles).  Both
// are within ~1 ulp of fp32, far below the bf16 rounding that follows (a different bf16 result
// only when the fp32 value sits within ~1.5 fp32 ulp of a bf16 rounding boundary).
__device__ __forceinline__ float silu_f(float g) {
  return g * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-g * 1.44269504088896341f));
}

// sum over the 16 lanes of a DPP row (lanes 16k .. 16k+15), in every lane: rotations by 8, 4,
// 2, 1 (row_ror DPP moves, no LDS); a fixed tree, so the result is deterministic
__device__ __forceinline__ float row16_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x124, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x122, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x121, 0xF, 0xF, false));
  return v;
}

// ============================================================ decode (M <= 64) kernel
// RMSNorm modes of the decode GEMV (NORM template argument, kernels.h DN_*):
//  DN_NONE  A used as is;
//  DN_EXACT Qwen3RMSNorm at the reference rounding points (qwen3_server_module.py:19-25):
//           A' = bf16(w * bf16(A * r)), r = 1 / sqrt(ssq[row] / K + eps) from the SSQ slot
//           the producer filled (ssq_out below; kernels.h DecodeNorm), applied to each A
//           fragment before its MFMA.
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
  // to part[y][row][col] (row stride ldp).
  float* part;
  int64_t ldp;
  // DN_EXACT: the SSQ slot (kernels.h DecodeNorm) holding A's row sums of squares, and the
  // norm weight [K]
  const unsigned long long* ssq_in;
  const u16* norm_w;
  // EPI_RESID producer side: the SSQ slot that receives the row sums of squares of the stored
  // bf16 outputs (the next DN_EXACT consumer's ssq_in), or null
  unsigned long long* ssq_out;
  // GEMM_PACK_A / GEMM_PACK_C (launch_gemm `pack`): A read / EPI_SILU output written
  // fragment-packed (packed_index); decode path only
  int pack;
  // EPI_SILU over a column range of the [gate; up] weight (a pipeline stage boundary inside a
  // layer's gate/up projection): 16-column tiles from a gate tile to its up tile (0: n_tiles,
  // the whole projection)
  int up_tiles;
};


// Row sums of squares between a decode producer and its DN_EXACT consumer (kernels.h DecodeNorm):
// q (>= 0, a 16-column tile's fp32 sum of squares of bf16 values) as the fixed-point pair
// hi = floor(q * 2^8), lo = frac(q * 2^8) * 2^32, added to one shard of the slot by no-return
// agent-scope 64-bit atomics (performed at the memory side: every XCD adds to the same words).
// Integer adds commute, so the slot's sum is the same whatever order the 256 producer workgroups
// arrive in.  q >= 2^47 (|x| > 3e6 in bf16 rows) or NaN saturates: the reference's fp32 sum
// would be as meaningless.  A workgroup adds its 16 rows' hi words and lo words with ONE wave
// instruction (lanes 0-15 hi, 16-31 lo: two contiguous 128-B runs), i.e. four 64-B atomic
// requests; the memory side serialises requests per 64-B segment, so 32 such per segment (one
// per shard member) instead of 8 per workgroup when each row went alone (+4 us per o GEMV).
__device__ __forceinline__ unsigned long long ssq_fixed(float q, bool lo_half) {
  float t = q * 256.0f;
  t = t < 3.6028797e16f ? t : 3.6028797e16f;  // 2^55 (also maps NaN here)
  const float ft = floorf(t);
  return lo_half ? (unsigned long long)(unsigned)((t - ft) * 4294967296.0f) : (unsigned long long)ft;
}
// the sum of a row's shards (hi0, lo0: this lane's two shards, summed; the wave's four 16-lane
// groups hold the other six) -> r = 1 / sqrt(sum / K + eps), in every lane of the row
__device__ __forceinline__ float ssq_rscale(unsigned long long hi, unsigned long long lo, int K, float eps) {
#pragma unroll
  for (int o = 16; o < 64; o <<= 1) {
    hi += __shfl_xor(hi, o);
    lo += __shfl_xor(lo, o);
  }
  const double tot = (double)hi * (1.0 / 256.0) + (double)lo * (1.0 / 1099511627776.0);
  return 1.0f / sqrtf((float)tot / (float)K + eps);
}

template <int NW, int NORM>
constexpr int decode_threads() {
  return NW * 64;
}

// dynamic LDS of a DN_EXACT workgroup over KT 32-column steps: per wave the staged bf16 norm
// weight of its batches, its fp32 copy in one-stream kernels, and the staged SSQ pieces
template <int NW, int TW>
__host__ __device__ constexpr int dn_region_bytes(int KT) {
  return ((KT / TW + NW - 1) / NW * TW * 4 + 63) / 64 * 1024;
}
template <int NORM, int S, int NW, int TW, int MT>
constexpr unsigned dn_lds_bytes(int KT) {
  return NORM == DN_EXACT ? (unsigned)(NW * (dn_region_bytes<NW, TW>(KT) * (S == 1 ? 3 : 1) + MT * 2048)) : 0u;
}

// APK: A is read fragment-packed (common.h packed_index: the decode path's act buffer, attention
// output and residual stream); the epilogue's R / C addressing follows g.pack at run time.
template <int MT, int S, int NW, int TW, int D, int EPI, int NORM, bool APK = false>
__global__ __launch_bounds__((decode_threads<NW, NORM>())) void gemm_decode_kernel(DecodeArgs g) {
  constexpr int NV = S * MT * 64;  // f32x4 values of one workgroup result
  __shared__ f32x4 red[NW][NV];
  // DN_EXACT (dynamic LDS, dn_lds_bytes): each wave stages the norm weight of its own batches
  // only (so no wave waits for another before its ring): bf16 as loaded (nstage, 1 KiB per 64
  // pieces), and for one-stream kernels an fp32 copy (nstage_f: saves the streaming waves one
  // unpack per element; the two-stream kernels amortise the unpack over two MFMAs)
  extern __shared__ __attribute__((aligned(16))) float dn_lds[];
  constexpr bool W_F32 = S == 1;
  const int M = g.M;
  const int nt = blockIdx.x;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  // K range of this workgroup (all of K unless EPI_PARTIAL splits it over gridDim.y)
  const int kt0 = (EPI == EPI_PARTIAL) ? (int)blockIdx.y * (g.KT / (int)gridDim.y) : 0;
  const int KT = (EPI == EPI_PARTIAL) ? g.KT / (int)gridDim.y : g.KT;
  // Two ring forms.  The exact-norm kernels (PADDED) load through buffer descriptors: a batch
  // index past the wave's last batch becomes an out-of-range offset (the load returns zeros),
  // every step issues unconditionally and the loop runs whole passes of straight-line code, so
  // hipcc's waitcnt pass counts exactly (a conditional issue makes it merge the issued and
  // not-issued paths and wait with the smallest count: with the norm wave's barriers in the
  // same kernel that drained the ring every pass, 14.55 -> 14.19 us for the Qwen3-8B q/k/v).
  // The other kernels keep global loads with the issue guarded: out-of-range loads are not
  // free (padding their short streams to whole passes cost 10-25 %: o 8.8 -> 10.1 us,
  // lm_head 232 -> 287 us), and there the merged waits cost less than the padding.
  const bf16x8* w0 = (const bf16x8*)(g.Wp + ((int64_t)nt * g.KT + kt0) * 512) + lane;
  const int up_dist = g.up_tiles ? g.up_tiles : g.n_tiles;  // [gate; up]: 16-column tiles from gate to up
  const bf16x8* w1 = (const bf16x8*)(g.Wp + ((int64_t)(nt + up_dist) * g.KT + kt0) * 512) + lane;
  const u16* a[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    int row = mt * 16 + (lane & 15);
    row = row < M ? row : M - 1;  // rows >= M compute garbage that is never stored
    a[mt] = APK ? g.A + ((int64_t)(mt * g.KT + kt0) * 64 + lane) * 8
                : g.A + (int64_t)row * g.lda + 8 * (lane >> 4) + kt0 * 32;
  }
  const __amdgpu_buffer_rsrc_t w0r = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(g.Wp + ((int64_t)nt * g.KT + kt0) * 512), 0, KT * 1024, 0x00020000);
  const __amdgpu_buffer_rsrc_t w1r = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(g.Wp + ((int64_t)(nt + up_dist) * g.KT + kt0) * 512), 0, KT * 1024, 0x00020000);
  const __amdgpu_buffer_rsrc_t ar = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(g.A + kt0 * (APK ? 512 : 32)), 0,
      APK ? (int)(((int64_t)(MT - 1) * g.KT + KT) * 1024) : (int)(((int64_t)(M - 1) * g.lda + KT * 32) * 2),
      0x00020000);
  int a_off[MT];  // byte offset of this lane's A fragment (k step 0) from ar
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    int row = mt * 16 + (lane & 15);
    row = row < M ? row : M - 1;  // rows >= M compute garbage that is never stored
    a_off[mt] = APK ? (int)((int64_t)mt * g.KT * 1024 + lane * 16) : (int)(((int64_t)row * g.lda + 8 * (lane >> 4)) * 2);
  }
  constexpr int OOB = 0x40000000;  // beyond every descriptor's range
  f32x4 acc[S][MT];
#pragma unroll
  for (int s = 0; s < S; ++s)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[s][mt] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nb = KT / TW;  // batches (the dispatcher guarantees KT % TW == 0)
  const int swave = __builtin_amdgcn_readfirstlane(wave);
  int b = swave;
  // this wave's batches b, b + NW, ... < nb
  const int nbw = swave < nb ? (nb - swave + NW - 1) / NW : 0;
  // DN_EXACT staging regions: dn_region_bytes(KT) per wave (whole KiB: a DMA instruction writes
  // 64 pieces), bf16 then (W_F32) the fp32 copy at twice the stride
  const int rgn = dn_region_bytes<NW, TW>(KT);
  char* const nssq = (char*)dn_lds + NW * rgn * (S == 1 ? 3 : 1) + swave * MT * 2048;  // [MT][8][2][16] u64
  u16* const nstage = (u16*)((char*)dn_lds + swave * rgn);
  float* const nstage_f = (float*)((char*)dn_lds + NW * rgn + swave * 2 * rgn);
  bf16x8 wv[D][S][TW], av[D][TW][MT];
  // DN_EXACT: a stage's activation fragments are issued BEFORE its weights, so the
  // normalisation of A can run as soon as A (L2) lands, while the weight bytes (HBM) are
  // still in flight (vmcnt retires in issue order)
  constexpr bool A_FIRST = NORM == DN_EXACT;
  // the lm_head GEMV (EPI_ARGMAX, 4 batches per wave) keeps the guarded ring with the exact norm
  // too: its padded passes would issue 2 dead batches per 4 live ones
  constexpr bool PADDED = NORM == DN_EXACT && EPI != EPI_ARGMAX;
  constexpr bool FULL_PROLOGUE = PADDED;
  constexpr int AKS = APK ? 512 : 32;  // elements between consecutive k-tiles of one lane's A
  constexpr int AKB = 2 * AKS;         // the same in bytes (buffer-load offsets)
  auto issue = [&](auto stage, int bb) {
    constexpr int d = decltype(stage)::value;
    if constexpr (!PADDED) {
      if constexpr (A_FIRST) {
#pragma unroll
        for (int u = 0; u < TW; ++u)
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) av[d][u][mt] = *(const bf16x8*)(a[mt] + (bb * TW + u) * AKS);
      }
#pragma unroll
      for (int u = 0; u < TW; ++u) {
        wv[d][0][u] = __builtin_nontemporal_load(w0 + (bb * TW + u) * 64);
        if constexpr (S == 2) wv[d][1][u] = __builtin_nontemporal_load(w1 + (bb * TW + u) * 64);
      }
      if constexpr (!A_FIRST) {
#pragma unroll
        for (int u = 0; u < TW; ++u)
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) av[d][u][mt] = *(const bf16x8*)(a[mt] + (bb * TW + u) * AKS);
      }
      return;
    }
    const bool live = bb < nb;
    const int wo = (live ? bb * TW * 1024 : OOB) + lane * 16;
    const int ao = live ? bb * TW * AKB : OOB;
    auto load_a = [&]() {
#pragma unroll
      for (int u = 0; u < TW; ++u)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
          av[d][u][mt] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(ar, a_off[mt] + ao + u * AKB, 0, 0));
    };
    if constexpr (A_FIRST) load_a();
#pragma unroll
    for (int u = 0; u < TW; ++u) {  // weights: nt (read once per step)
      wv[d][0][u] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(w0r, wo + u * 1024, 0, 2));
      if constexpr (S == 2)
        wv[d][1][u] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(w1r, wo + u * 1024, 0, 2));
    }
    if constexpr (!A_FIRST) load_a();
    // stages stay in issue order (the prologue's too: the loop's counted waits assume it)
    __builtin_amdgcn_sched_barrier(0);
  };
  static_assert(!FULL_PROLOGUE || PADDED, "the full prologue issues unguarded");
  // EPI_RESID: the residual elements this thread's epilogue adds (thread p < MT*64: rows
  // mt*16 + 4*(ln>>4) + r, column nt*16 + (ln&15)), loaded before the weight stream so the
  // epilogue at the kernel's tail does not wait a memory round trip for them
  u16 rpre[4] = {0, 0, 0, 0};
  if constexpr (EPI == EPI_RESID) {
    const int p = threadIdx.x;
    if (p < MT * 64) {
      const int mt = p >> 6, ln = p & 63;
      const int col = nt * 16 + (ln & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = mt * 16 + 4 * (ln >> 4) + r;
        if (row < M)
          rpre[r] = g.R[(g.pack & GEMM_PACK_R) ? packed_index(row, col, g.ldr) : (int64_t)row * g.ldr + col];
      }
    }
  }
  float rr[MT];  // DN_EXACT: r of row mt*16 + (lane & 15)
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) rr[mt] = 1.0f;
  if constexpr (NORM == DN_EXACT) {
    if (nbw > 0) {
      // Issued before the weight prologue, so the waits for them are counted (vmcnt retires in
      // issue order) and never drain the ring: (1) the row sums of squares, lane l reading shards
      // 2(l/16), 2(l/16)+1 of row mt*16 + l%16; (2) the norm weight of this wave's own batches by
      // LDS-DMA into the wave's staging region (no registers): 16-B piece p = 64i + lane is
      // batch j = p / (4TW) of the wave, columns 8(p % (4TW)) on, so a step's fragment sits at
      // (j TW + u) 32 + 8(lane / 16) of the region, like the global columns with b -> j
      typedef __attribute__((address_space(3))) void* lds_ptr;
      {
        // (1) by LDS-DMA too (no registers held across the prologue): piece (mt, h) of lane l
        // to the wave's ssq area at ((mt * 2 + h) * 64 + l) * 16
        const __amdgpu_buffer_rsrc_t sr =
            __builtin_amdgcn_make_buffer_rsrc((void*)g.ssq_in, 0, SSQ_SLOT_WORDS * 8, 0x00020000);
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int k = 0; k < 2; ++k) {
            // 128-B run c = (shard, hi|lo) of rows mt*16.. -> LDS [shard][hi|lo][16 rows] u64
            const int c = (64 * k + lane) >> 3;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(sr, (lds_ptr)(nssq + mt * 2048 + k * 1024), 16,
                                                     (c * 64 + mt * 16) * 8 + (lane & 7) * 16, 0, 0, 0);
          }
      }
      {
        const __amdgpu_buffer_rsrc_t nr =
            __builtin_amdgcn_make_buffer_rsrc((void*)(g.norm_w + kt0 * 32), 0, KT * 64, 0x00020000);
        const int npieces = nbw * TW * 4;
        for (int i = 0; i * 64 < npieces; ++i) {  // wave-uniform trip count
          const int p = 64 * i + lane;
          const int j = p / (4 * TW), c = p % (4 * TW);
          const int col = ((swave + j * NW) * TW) * 32 + 8 * c;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(nr, (lds_ptr)(nstage + i * 512), 16,
                                                   p < npieces ? col * 2 : OOB, 0, 0, 0);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      // the staged row sums and norm weight have landed once every load but the prologue's has
      // retired
      if constexpr (PADDED) {  // prologue: all D stages
        [&]<int... I>(std::integer_sequence<int, I...>) {
          (issue(std::integral_constant<int, I>{}, b + I * NW), ...);
        }(std::make_integer_sequence<int, D>{});
        vm_wait<D * TW * (MT + S)>();
      } else {  // stages 0..D-2, guarded
        [&]<int... I>(std::integer_sequence<int, I...>) {
          ((b + I * NW < nb ? issue(std::integral_constant<int, I>{}, b + I * NW) : void()), ...);
        }(std::make_integer_sequence<int, D - 1>{});
        if (nbw >= D - 1)
          vm_wait<(D - 1) * TW * (MT + S)>();
        else
          vm_wait<0>();
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        // lane l: row l % 16, shards 2(l / 16) and 2(l / 16) + 1
        const unsigned long long* w =
            (const unsigned long long*)(nssq + mt * 2048) + (4 * (lane >> 4)) * 16 + (lane & 15);
        rr[mt] = ssq_rscale(w[0] + w[32], w[16] + w[48], g.KT * 32, g.eps);
      }
      if constexpr (W_F32) {
        for (int p = lane; p < nbw * TW * 4; p += 64) {
          const u16x8 nv = *(const u16x8*)(nstage + p * 8);
          f32x4 lo, hi;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            lo[j] = bf2f(nv[j]);
            hi[j] = bf2f(nv[4 + j]);
          }
          *(f32x4*)(nstage_f + p * 8) = lo;
          *(f32x4*)(nstage_f + p * 8 + 4) = hi;
        }
      }
    }
  } else if (nbw > 0) {
    // prologue: stages 0..D-2 (all D with FULL_PROLOGUE)
    [&]<int... I>(std::integer_sequence<int, I...>) {
      ((PADDED || b + I * NW < nb ? issue(std::integral_constant<int, I>{}, b + I * NW) : void()), ...);
    }(std::make_integer_sequence<int, FULL_PROLOGUE ? D : D - 1>{});
  }
  if (nbw > 0) {
    // one step: issue the batch D-1 steps ahead into the slot this step's predecessor freed,
    // then consume slot d.  With FULL_PROLOGUE the first step's issue went out with the
    // prologue, so that step is peeled (no issue) and the loop runs the slots rotated by one
    bool fin = false;
    auto step = [&](auto stage, auto may_issue) {
      constexpr int d = decltype(stage)::value;
      if constexpr (!PADDED) {
        if (fin) return;
        const int nxt = b + (D - 1) * NW;
        if (nxt < nb) issue(std::integral_constant<int, (d + D - 1) % D>{}, nxt);
      } else if constexpr (decltype(may_issue)::value) {
        issue(std::integral_constant<int, (d + D - 1) % D>{}, b + (D - 1) * NW);
      }
      // keep the issued loads ahead of the MFMAs (the scheduler would otherwise
      // interleave them to save registers, leaving few loads in flight)
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (NORM == DN_EXACT) {
#pragma unroll
        for (int u = 0; u < TW; ++u) {
          // steps past the wave's last batch (zeros from their loads) re-read its last batch's
          // weight: finite, so 0 * w stays 0
          const int wo = (min((b - swave) / NW, nbw - 1) * TW + u) * 32 + 8 * (lane >> 4);
          float wf[8];
          if constexpr (W_F32) {
            const f32x4 w_lo = *(const f32x4*)(nstage_f + wo), w_hi = *(const f32x4*)(nstage_f + wo + 4);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              wf[j] = w_lo[j];
              wf[4 + j] = w_hi[j];
            }
          } else {
            const u16x8 nv = *(const u16x8*)(nstage + wo);
#pragma unroll
            for (int j = 0; j < 8; ++j) wf[j] = bf2f(nv[j]);
          }
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) {
            const u16x8 xv = __builtin_bit_cast(u16x8, av[d][u][mt]);
            bf16x8 y;
#pragma unroll
            for (int j = 0; j < 8; ++j) y[j] = (__bf16)(wf[j] * rbf(bf2f(xv[j]) * rr[mt]));
            av[d][u][mt] = y;
          }
        }
      }
#pragma unroll
      for (int u = 0; u < TW; ++u)
#pragma unroll
        for (int s = 0; s < S; ++s)
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) acc[s][mt] = mfma16(av[d][u][mt], wv[d][s][u], acc[s][mt]);
      __builtin_amdgcn_sched_barrier(0);
      b += NW;
      if (b >= nb) fin = true;
    };
    constexpr int R = FULL_PROLOGUE ? 1 : 0;  // slot rotation of the loop body
    if constexpr (FULL_PROLOGUE) step(std::integral_constant<int, 0>{}, std::false_type{});
    if constexpr (PADDED) {
      // whole passes; steps past the wave's last batch consume the zeros their loads returned
      for (int pass = (nbw - R + D - 1) / D; pass > 0; --pass) {
        [&]<int... I>(std::integer_sequence<int, I...>) {
          (step(std::integral_constant<int, (I + R) % D>{}, std::true_type{}), ...);
        }(std::make_integer_sequence<int, D>{});
      }
    } else {
      while (!fin) {
        [&]<int... I>(std::integer_sequence<int, I...>) {
          (step(std::integral_constant<int, I>{}, std::true_type{}), ...);
        }(std::make_integer_sequence<int, D>{});
      }
    }
  }
  {
#pragma unroll
    for (int s = 0; s < S; ++s)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) red[wave][(s * MT + mt) * 64 + lane] = acc[s][mt];
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
    }
    return;
  }
  float qr[4] = {0.f, 0.f, 0.f, 0.f};  // EPI_RESID: the tile's sums of squares of rows 4(ln/16)+r
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
    } else if constexpr (EPI == EPI_RESID) {
      // all lanes take part in the 16-lane ssq reduction: rows >= M contribute zero
      const bool live = row < M;
      const u16 ob = live ? f2bf(rbf(v[0][r]) + bf2f(rpre[r])) : (u16)0;
      if (live) g.C[(g.pack & GEMM_PACK_C) ? packed_index(row, col, g.ldc) : (int64_t)row * g.ldc + col] = ob;
      if (g.ssq_out) qr[r] = row16_sum(bf2f(ob) * bf2f(ob));
    } else if (row < M) {
      float o;
      if constexpr (EPI == EPI_NONE) {
        o = v[0][r];
      } else if constexpr (EPI == EPI_SILU) {
        o = rbf(silu_f(rbf(v[0][r]))) * rbf(v[S - 1][r]);
      } else {
        o = 0.f;  // EPI_PARTIAL returns above
      }
      g.C[(g.pack & GEMM_PACK_C) ? packed_index(row, col, g.ldc) : (int64_t)row * g.ldc + col] = f2bf(o);
    }
  }
  if constexpr (EPI == EPI_RESID) {
    if (g.ssq_out) {
      // lane i < 32 takes row i % 16 (held by lanes 16(i%16 / 4) .. as qr[i % 4]) and adds its hi
      // (i < 16) or lo word to shard nt % SSQ_SHARDS: slot [shard][hi | lo][64 rows]
      const int i = ln & 15;
      float qv = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float t = __shfl(qr[r], 16 * (i >> 2));
        if ((i & 3) == r) qv = t;
      }
      const int row = mt * 16 + i;
      if (ln < 32 && row < M)
        __hip_atomic_fetch_add(g.ssq_out + (nt % SSQ_SHARDS) * 128 + (ln >> 4) * 64 + row, ssq_fixed(qv, ln >= 16),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ring shape per (row tiles, streams): tuned on the Qwen3-8B decode shapes (tools/gemv_lab.hip)
// Round 4 re-sweep of the one-stream, one-row-tile shape (tools/decode_lib_ab.sh, eager event
// means, one box): D = 4 takes the o GEMV (K = 4096, four batches per wave) from 11.4 to 10.9 us,
// but the lm_head GEMV from 214 to 239 us and down from 22.1 to 22.3; D = 5, TW = 2 / D = 4 and
// TW = 8 / D = 2 were slower in the step.  So D = 4 only for short-K residual GEMVs (DecodeShortK).
// Also slower: the q/k/v partial GEMV at D = 4 (14.9 -> 16.6 us) and the gate/up GEMV at D = 3
// (35.3 -> 37.2 us); the q/k/v one at D = 2 changed nothing.
template <int MT, int S>
struct DecodeCfg {
  static constexpr int NW = S == 1 ? 8 : 4;
  static constexpr int TW = (MT <= 2) ? 4 : 2;
  static constexpr int D = (S == 1 && MT == 1) ? 3 : 2;
};
constexpr int DECODE_SHORT_KT = 128;  // K <= 4096: the whole K range is <= 4 batches per wave

template <int MT, int EPI, int NORM>
static void decode_launch(const DecodeArgs& a, hipStream_t s) {
  constexpr int S = (EPI == EPI_SILU) ? 2 : 1;
  using C = DecodeCfg<MT, S>;
  constexpr int T = decode_threads<C::NW, NORM>();
  if constexpr (S == 1 && MT == 1 && EPI == EPI_RESID) {  // short K: one more batch in flight
    if (a.KT <= DECODE_SHORT_KT && a.KT % C::TW == 0) {
      if (a.pack & GEMM_PACK_A)
        hipLaunchKernelGGL((gemm_decode_kernel<MT, S, C::NW, C::TW, 4, EPI, NORM, true>), dim3(a.n_tiles), dim3(T),
                           (dn_lds_bytes<NORM, S, C::NW, C::TW, MT>(a.KT)), s, a);
      else
        hipLaunchKernelGGL((gemm_decode_kernel<MT, S, C::NW, C::TW, 4, EPI, NORM>), dim3(a.n_tiles), dim3(T),
                           (dn_lds_bytes<NORM, S, C::NW, C::TW, MT>(a.KT)), s, a);
      return;
    }
  }
  if (a.pack & GEMM_PACK_A) {
    if (a.KT % C::TW == 0)
      hipLaunchKernelGGL((gemm_decode_kernel<MT, S, C::NW, C::TW, C::D, EPI, NORM, true>), dim3(a.n_tiles), dim3(T),
                         (dn_lds_bytes<NORM, S, C::NW, C::TW, MT>(a.KT)), s, a);
    else
      hipLaunchKernelGGL((gemm_decode_kernel<MT, S, C::NW, 1, 2, EPI, NORM, true>), dim3(a.n_tiles), dim3(T),
                         (dn_lds_bytes<NORM, S, C::NW, 1, MT>(a.KT)), s, a);
    return;
  }
  if (a.KT % C::TW == 0)
    hipLaunchKernelGGL((gemm_decode_kernel<MT, S, C::NW, C::TW, C::D, EPI, NORM>), dim3(a.n_tiles), dim3(T),
                       (dn_lds_bytes<NORM, S, C::NW, C::TW, MT>(a.KT)), s, a);
  else  // odd K/32 (single-op API only; every Qwen3 projection has K % 128 == 0)
    hipLaunchKernelGGL((gemm_decode_kernel<MT, S, C::NW, 1, 2, EPI, NORM>), dim3(a.n_tiles), dim3(T),
                       (dn_lds_bytes<NORM, S, C::NW, 1, MT>(a.KT)), s, a);
}

template <int EPI, int NORM>
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
// reduction left to the consumer (launch_attn_decode_fused): with NW = 4 the 384 x 2
// workgroups of Qwen3-8B sit 3 per CU, every CU streaming the same bytes.  `norm` selects
// the RMSNorm mode: DN_EXACT (ssq slot / norm_w) or none.
void launch_gemm_decode_partial(const u16* A, int64_t lda, const u16* Wp, int M, int N, int K, int kslices,
                                float* part, const DecodeNorm& norm, hipStream_t s, int pack) {
  DecodeArgs a = {};
  a.A = A;
  a.lda = lda;
  a.Wp = Wp;
  a.KT = K / 32;
  a.n_tiles = N / 16;
  a.M = M;
  a.eps = norm.eps;
  a.part = part;
  a.ldp = N;
  a.ssq_in = norm.ssq;
  a.norm_w = norm.w;
  a.pack = pack;
  const dim3 grid(N / 16, kslices);
  if (norm.mode == DN_EXACT && (pack & GEMM_PACK_A))
    hipLaunchKernelGGL((gemm_decode_kernel<1, 1, 4, 4, 3, EPI_PARTIAL, DN_EXACT, true>), grid,
                       dim3(decode_threads<4, DN_EXACT>()), (dn_lds_bytes<DN_EXACT, 1, 4, 4, 1>(a.KT / kslices)), s, a);
  else if (norm.mode == DN_EXACT)
    hipLaunchKernelGGL((gemm_decode_kernel<1, 1, 4, 4, 3, EPI_PARTIAL, DN_EXACT>), grid,
                       dim3(decode_threads<4, DN_EXACT>()), (dn_lds_bytes<DN_EXACT, 1, 4, 4, 1>(a.KT / kslices)), s, a);
  else
    hipLaunchKernelGGL((gemm_decode_kernel<1, 1, 4, 4, 3, EPI_PARTIAL, DN_NONE>), grid, dim3(256), 0, s, a);
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
    // (the split slices first instead, so the publishing CUs take whole tiles while the
    // combining ones finish: no change, o 534.4 vs 534.4 us, round 4)
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
  // row-group depth: 8 row blocks up to 8192 rows (M <= 16383), 4 beyond.  Per-shape A/Bs of the
  // 32B projections (profiles/r05/gemm_gm_ab*.txt): at M = 32768 (config 5, B = 4) GM = 4 ran
  // gate/up 6.8 %, q/k/v 4.8 %, down 1.2 % faster than 8 (A = 335 MB no longer stays in the
  // Infinity Cache, so shallower groups keep each XCD's A panels hot); at M = 8192 within 0-2 %.
#ifdef W4_GM
  constexpr int GM = W4_GM;  // lab builds pin it (tools/build_probes.sh)
#else
  const int GM = grid_m >= 64 ? 4 : 8;
#endif
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


// Tail-split partials: slice sl of split tile sidx is 65536 fp32 at ws + (sidx * nsl + sl) *
// 65536; accumulator tile (i, j) of thread x is the 16 bytes at ((i * 8 + j) * 256 + x) (one
// 1 KiB run per wave store).  The publisher stores straight from the accumulator AGPRs
// (global_store_dwordx4 with an AGPR source, sc1: write-through to the coherence point), so no
// accumulator is copied to VGPRs; the combiner, after an agent-scope acquire, reads them with
// plain loads in its epilogue and sums over the slices in slice order (two slices: p0 + p1, the
// same bits whichever slice combines).
__device__ __forceinline__ void split_publish(const f32x4 (&acc)[8][8], float* part, int slice) {
  f32x4* dst = (f32x4*)(part + (size_t)slice * 65536) + threadIdx.x;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j)
      asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(dst + (i * 8 + j) * 256), "a"(acc[i][j]) : "memory");
}

__device__ __forceinline__ f32x4 split_tile_sum(const f32x4& mine, const float* part, int nsl, int slice, int i,
                                                int j) {
  const f32x4* src = (const f32x4*)part + (i * 8 + j) * 256 + threadIdx.x;
  if (nsl == 2) return mine + src[(size_t)(1 - slice) * 16384];
  f32x4 sum = {0.f, 0.f, 0.f, 0.f};
  for (int sl = 0; sl < nsl; ++sl) {
    const f32x4 l = src[(size_t)sl * 16384];
    sum += (sl == slice) ? mine : l;
  }
  return sum;
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
template <int EPI>
__global__ __launch_bounds__(256, 1) void gemm_w4_kernel(
    const u16* __restrict__ A, int64_t lda, const u16* __restrict__ Wp, int KT, int n_tiles_w,
    u16* __restrict__ C, int64_t ldc, const u16* __restrict__ R, int64_t ldr, int M, int grid_m, int grid_n,
    SplitTail st) {
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
  // buffer_load_dwordx4 ... lds with the per-piece and per-step offsets in SGPRs (soffset)
  // instead of a 64-bit VGPR address per piece
  const __amdgpu_buffer_rsrc_t a_rsrc =
      __builtin_amdgcn_make_buffer_rsrc((void*)a_base, 0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t b_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)Wp, 0, 0x7fffffff, 0x00020000);
  auto issue = [&](int p, int t, int buf) {  // piece p (0-7 A, 8-15 B) of K-step t into buffer buf
    char* base = lds + buf * 65536;
    typedef __attribute__((address_space(3))) void* lds_ptr;
    if (p < 8)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(a_rsrc, (lds_ptr)(base + (8 * wv + p) * 1024), 16, a_voff[p], t * 128,
                                               0, 0);
    else
      __builtin_amdgcn_raw_ptr_buffer_load_lds(b_rsrc, (lds_ptr)(base + 32768 + (8 * wv + p - 8) * 1024), 16, b_voff,
                                               (int)(b_soff[p - 8] + (int64_t)t * 2048), 0, 0);
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
  // rows 0-63, [C] F1 rows 64-127
  auto mfx = [&](int x) {
    const int kh = (x >= 64) ? 1 : 0;
    const int q = x & 31, half = (x >> 5) & 1;  // group of 32: rows 64 * half + ...
    mf(kh, 4 * half + (q & 3), q >> 2);  // nt-major inside each group of 32
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

  float* part = nsl > 1 ? st.ws + (size_t)sidx * nsl * 65536 : nullptr;
  auto tile_sum = [&](int i, int j) -> f32x4 {
    return nsl > 1 ? split_tile_sum(acc[i][j], part, nsl, slice, i, j) : acc[i][j];
  };
  if (nsl > 1) {  // ---- tail split: publish or combine (tools/archive/gemm_superseded.hip had the same in the 8-wave ring)
    __syncthreads();
    unsigned* ticket_lds = (unsigned*)lds;
    unsigned* cnt = st.cnt + sidx;
    unsigned* done = st.cnt + 8 * (st.tiles_per_xcd - st.full_per_xcd) + sidx;
    if (threadIdx.x == 0) ticket_lds[0] = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const unsigned ticket = ticket_lds[0];
    if (ticket + 1 < (unsigned)nsl) {
      // Hand-off form (MI355X_MICROARCH.md, "Valid forms besides Guideline 16's R1/R2", the
      // producer's write-through variant): every partial is an sc1 (write-through) store, every
      // storing wave waits vmcnt(0), a barrier, then a relaxed agent-scope add; the combiner
      // polls relaxed, then one agent acquire fence before its loads.  A C++ __ATOMIC_RELEASE add
      // would compile to an extra buffer_wbl2 sc1 (~1.7 us, nothing is dirty: the stores are
      // write-through) and an __ATOMIC_ACQUIRE poll to a buffer_inv per iteration on gfx950 (hipcc
      // -S, round 5), so the guide's form is kept; the inline-asm wait is not visible to the
      // compiler's waitcnt pass, so nothing can drop it (the guide's "Compiler hazard").
      split_publish(acc, part, slice);
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
    // acquire (L1 / non-coherent L2 lines invalidated); the epilogue adds the other slices'
    // partials with plain loads (relaxed atomic loads were issued one round trip at a time:
    // tools/w4_stamps.py measured 54 us of combine for 256 KiB)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }

  // ---- epilogue: lane holds C[row = ... + (lane & 15)][col = ... + 4 * (lane >> 4) + r]
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = m0 + wr * 128 + i * 16 + (lane & 15);
    if (row >= M) continue;
    if constexpr (EPI == EPI_SILU) {
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const int col = n0 + wc * 64 + nt * 16 + 4 * (lane >> 4);
        u16x4 v;
        const f32x4 g4 = tile_sum(i, nt), u4 = tile_sum(i, 4 + nt);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float gg = rbf(g4[r]);
          const float uu = rbf(u4[r]);
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
        const f32x4 a4 = tile_sum(i, j);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float o = a4[r];
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
                                             int lane) {
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
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = row0 + 16 * i + (lane & 15);
      const int rowc = row < M ? row : M - 1;
      pos[i] = e.positions[rowc];
      slot[i] = isq ? 0 : e.slots[rowc];
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
      float x[8][4];
      float ss = 0.f;
#pragma unroll
      for (int nt = 0; nt < 8; ++nt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          x[nt][r] = rbf(acc[i][nt][r]);  // the bf16 projection output
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
#pragma unroll
    for (int i = 0; i < 8; ++i) slots[i] = e.slots[min(row0 + 16 * i + (lane & 15), M - 1)];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = row0 + 16 * i + (lane & 15);
      if (row >= M) continue;
      const int slot = slots[i];
      if (slot < 0) continue;
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
          blk[((kt * 8 + nt) * 64 + ln) * 8 + jj] = f2bf(acc[i][nt][r]);
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
// units.  Whole tiles only: grids that need the tail split run gemm_w4_kernel (the split
// inside this loop, as a separate instantiation, spilled 60 VGPRs and ran o / down 2-4 %
// slower than gemm_w4_kernel's: tools/gemm_bench.py A/B, round 4).
template <int EPI>
__global__ __launch_bounds__(256, 1) void gemm_w4p_kernel(
    const u16* __restrict__ A, int64_t lda, const u16* __restrict__ Wp, int KT, int n_tiles_w,
    u16* __restrict__ C, int64_t ldc, const u16* __restrict__ R, int64_t ldr, int M, int grid_m, int grid_n,
    SplitTail st, int nunits, QkvEpilogue qe) {
  __shared__ __attribute__((aligned(16))) char lds[2 * 65536 + 16];  // + the split ticket
  typedef __attribute__((address_space(3))) void* lds_ptr;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wr = wave >> 1, wc = wave & 1;
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  // vector-memory operations per wave in one epilogue
  constexpr int EPI_OPS = EPI == EPI_SILU ? 32 : EPI == EPI_RESID ? 128 : 64;
  const __amdgpu_buffer_rsrc_t c_rsrc =
      __builtin_amdgcn_make_buffer_rsrc((void*)C, 0, (int)((int64_t)M * ldc * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t r_rsrc =
      __builtin_amdgcn_make_buffer_rsrc((void*)R, 0, R ? (int)((int64_t)M * ldr * 2) : 0, 0x00020000);

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
    // the lane from opaque_lane() and the wave from its SGPR: what derives from them is
    // recomputed per unit instead of hoisted out of the persistent loop and kept live across the
    // K-loop (hipcc spilled those per-lane invariants in the EPI_QKV instantiation -- 35 VGPRs --
    // and reloaded them every unit behind vmcnt(0) waits)
    const int ln = opaque_lane();
    const int lda2 = (int)lda * 2;  // rr < 256 rows past the unit's base: 32-bit offsets
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      const int i = 64 * wv + 8 * p + (ln >> 3);  // image row 0..255
      const int rr = (u.m0 + i < M ? i : M - 1 - u.m0);
      const int chunk = (ln & 7) ^ ((i >> 1) & 7);
      a_voff[p] = (unsigned)(rr * lda2 + chunk * 16);
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
    // next tile's sources are then computed after the epilogue (fewer live registers in it).
    // Round 4 (tools/span_ab.py, tools/w4p_stamps.py): with the prefetch, -14 / -13 / +3 us
    // per 32B launch on three boxes; issuing the pieces inside the epilogue once its own loads
    // were in flight spilled into the K-loop (14x slower); V accumulated transposed for 8-byte
    // V^T stores and every cos/sin load issued up front: no change.  The epilogue's ~19 us per
    // unit (every CU at once) stays.
    constexpr bool XPF = EPI != EPI_QKV;
    if (has_next) {
      un = unit_of(vn);
      if constexpr (XPF) src_of(un);
    }
    iter(std::integral_constant<int, 1>{}, ZF{}, u.nK - 2, par, XPF && has_next);
    iter(std::integral_constant<int, 2>{}, ZF{}, u.nK - 1, par, XPF && has_next);
    acc_fence();

    if constexpr (EPI == EPI_QKV) {
      // opaque lane (src_of): the epilogue's per-lane addresses are computed here, not hoisted
      // across the K-loop (they were the other spills of this instantiation)
      qkv_epilogue(acc, qe, u.m0 + (wv >> 1) * 128, (u.n0 >> 7) + (wv & 1), M, opaque_lane());
    } else {  // ---- epilogue: lane holds C[row = ... + (lane & 15)][col = ... + 4 * (lane >> 4) + r]
      // buffer loads/stores: rows >= M are issued and dropped by the range check, so the
      // epilogue's vector-memory count is fixed (EPI_OPS) and the next unit's wait is exact
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int row = u.m0 + wr * 128 + i * 16 + (lane & 15);
        if constexpr (EPI == EPI_SILU) {
#pragma unroll
          for (int nt = 0; nt < 4; ++nt) {
            const int col = u.n0 + wc * 64 + nt * 16 + 4 * (lane >> 4);
            u16x4 o;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float gg = rbf(acc[i][nt][r]);
              const float uu = rbf(acc[i][4 + nt][r]);
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
              float x = acc[i][j][r];
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

static void w4_launch(int epi, int grid, hipStream_t s, const u16* A, int64_t lda, const u16* Wp, int KT, int ntw,
                      u16* C, int64_t ldc, const u16* R, int64_t ldr, int M, int gm, int gn, const SplitTail& st) {
  switch (epi) {
    case EPI_NONE:
      hipLaunchKernelGGL((gemm_w4_kernel<EPI_NONE>), dim3(grid), dim3(256), 0, s, A, lda, Wp, KT, ntw, C, ldc, R, ldr,
                         M, gm, gn, st);
      break;
    case EPI_RESID:
      hipLaunchKernelGGL((gemm_w4_kernel<EPI_RESID>), dim3(grid), dim3(256), 0, s, A, lda, Wp, KT, ntw, C, ldc, R,
                         ldr, M, gm, gn, st);
      break;
    default:
      hipLaunchKernelGGL((gemm_w4_kernel<EPI_SILU>), dim3(grid), dim3(256), 0, s, A, lda, Wp, KT, ntw, C, ldc, R,
                         ldr, M, gm, gn, st);
      break;
  }
}

// persistent grid: one workgroup per CU, a multiple of 8 (units keep their XCD), <= units
#define W4P_MAX_DEVICES 16
static int w4p_grid(int units) {
  static int ncu[W4P_MAX_DEVICES] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= W4P_MAX_DEVICES) dev = 0;
  if (ncu[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    ncu[dev] = n;
  }
  if (units <= ncu[dev]) return units;
  return ncu[dev] & ~7;
}

// The tail split's fixed maximum: each XCD cuts its last `rem` tiles into 32 / rem slices, so
// rem * split = 32 slices of a 256x256 fp32 tile per XCD, and 2 x 8 x rem <= 512 tickets.
#define SPLIT_WS_BYTES ((size_t)8 * 32 * 65536 * sizeof(float))
#define SPLIT_CNT_N 512

int gemm_ws_alloc(GemmWs* w) {
  if (!w->split) return hipSuccess;
  hipError_t e = hipMalloc((void**)&w->ws, SPLIT_WS_BYTES);
  if (e == hipSuccess) e = hipMalloc((void**)&w->cnt, SPLIT_CNT_N * sizeof(unsigned));
  if (e == hipSuccess) e = hipMemset(w->cnt, 0, SPLIT_CNT_N * sizeof(unsigned));
  return (int)e;
}

void gemm_ws_free(GemmWs* w) {
  if (!w) return;
  if (w->ws) (void)hipFree(w->ws);
  if (w->cnt) (void)hipFree(w->cnt);
  w->ws = nullptr;
  w->cnt = nullptr;
}

// Tail-split plan for `tiles` 256x256 tiles of nK K-steps on 8 XCDs x 32 CUs (one workgroup
// per CU), with its fp32 partials and tickets in the caller's (span's) preallocated workspace
// (no workspace, or split = 0: no split).  Nothing here allocates, so it is capture-safe.
static SplitTail plan_split_tail(int tiles, int nK, const GemmWs* w) {
  SplitTail st = {1, 0, 0, 0, nullptr, nullptr};
  if (!w || !w->split || !w->ws || !w->cnt) return st;
  if (tiles % 8) return st;
  const int per = tiles / 8, rem = per % 32;
  if (rem == 0 || 32 % rem) return st;
  const int split = 32 / rem;
  if (split > 8 || nK % split || nK / split < 3) return st;
  st.split = split;
  st.tiles_per_xcd = per;
  st.full_per_xcd = per - rem;
  st.units_per_xcd = per - rem + rem * split;
  st.ws = w->ws;
  st.cnt = w->cnt;
  return st;
}

// the 256x256 four-wave bodies (gemm_w4p / gemm_w4): >= 512 rows, whole 256-column tiles
static bool use_w4(int M, int N, int K, int epi) {
  if (M < 512 || K < 192) return false;
  return (epi == EPI_SILU) ? (N % 128 == 0) : (N % 256 == 0);
}

// ============================================================ dispatch
bool gemm_uses_tiled(int M, int N, int K, int epi) {
  return (M > 64) && (K % TBK == 0) && ((epi == EPI_SILU) ? (N % 64 == 0) : (N % TBN == 0)) &&
         epi != EPI_ARGMAX;
}

bool launch_gemm(const u16* A, int64_t lda, const u16* Wp, int M, int N, int K, u16* C, int64_t ldc,
                 const u16* R, int64_t ldr, int epi, unsigned long long* keys, hipStream_t s, const GemmWs* ws,
                 const DecodeNorm* dn, unsigned long long* ssq_out, int pack, int up_tiles) {
  const int KT = K / 32;
  const int n_tiles = N / 16;  // output tiles of 16 columns
  const bool tiled = gemm_uses_tiled(M, N, K, epi);
  if (up_tiles && (tiled || epi != EPI_SILU)) return false;  // column ranges: decode SwiGLU only
  if (tiled && use_w4(M, N, K, epi)) {
    const int ncols = (epi == EPI_SILU) ? 128 : 256;
    const int gm = (M + 255) / 256, gn = N / ncols;
    const int ntw = (epi == EPI_SILU) ? 2 * n_tiles : n_tiles;
    const SplitTail st = plan_split_tail(gm * gn, K / 64, ws);
    const int grid = st.split > 1 ? 8 * st.units_per_xcd : gm * gn;
    // w4p addresses C / R through 32-bit buffer offsets
    const bool fits32 = (int64_t)(M + 256) * ldc * 2 < 0x7fffffff && (!R || (int64_t)(M + 256) * ldr * 2 < 0x7fffffff);
    if (fits32 && st.split == 1) {
      const int g = w4p_grid(grid);
      switch (epi) {
        case EPI_NONE:
          hipLaunchKernelGGL(gemm_w4p_kernel<EPI_NONE>, dim3(g), dim3(256), 0, s, A, lda, Wp, KT, ntw, C, ldc, R, ldr,
                             M, gm, gn, st, grid, QkvEpilogue{});
          break;
        case EPI_RESID:
          hipLaunchKernelGGL(gemm_w4p_kernel<EPI_RESID>, dim3(g), dim3(256), 0, s, A, lda, Wp, KT, ntw, C, ldc, R, ldr,
                             M, gm, gn, st, grid, QkvEpilogue{});
          break;
        default:
          hipLaunchKernelGGL(gemm_w4p_kernel<EPI_SILU>, dim3(g), dim3(256), 0, s, A, lda, Wp, KT, ntw, C, ldc, R, ldr,
                             M, gm, gn, st, grid, QkvEpilogue{});
          break;
      }
      return true;
    }
    w4_launch(epi, grid, s, A, lda, Wp, KT, ntw, C, ldc, R, ldr, M, gm, gn, st);  // tail split
    return true;
  }
  if (tiled) {
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
    return true;
  }
  // decode path, 64-row slabs (M > 64 only when the tiled shape constraints fail).  The
  // DN_EXACT norm and the ssq_out partials are defined for M <= 64 only: refused (nothing
  // launched, false), so a consumer never reads a slot no producer filled
  const int mode = dn ? dn->mode : DN_NONE;
  if ((mode == DN_EXACT || ssq_out) && M > 64) return false;
  if (mode == DN_EXACT && epi == EPI_RESID) return false;  // no such body
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
    a.eps = dn ? dn->eps : 0.f;
    a.ssq_out = (epi == EPI_RESID) ? ssq_out : nullptr;
    a.pack = pack;
    a.up_tiles = up_tiles;
    if (mode == DN_EXACT) {
      a.ssq_in = dn->ssq;
      a.norm_w = dn->w;
      switch (epi) {
        case EPI_NONE: decode_mt<EPI_NONE, DN_EXACT>(a, s); break;
        case EPI_SILU: decode_mt<EPI_SILU, DN_EXACT>(a, s); break;
        default: decode_mt<EPI_ARGMAX, DN_EXACT>(a, s); break;
      }
    } else {
      switch (epi) {
        case EPI_NONE: decode_mt<EPI_NONE, DN_NONE>(a, s); break;
        case EPI_RESID: decode_mt<EPI_RESID, DN_NONE>(a, s); break;
        case EPI_SILU: decode_mt<EPI_SILU, DN_NONE>(a, s); break;
        default: decode_mt<EPI_ARGMAX, DN_NONE>(a, s); break;
      }
    }
    if (epi == EPI_ARGMAX) break;  // argmax requires M <= 64 (checked by the caller)
  }
  return true;
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

// The same reduction for a vocab-parallel lm_head shard (inferd_span_head_shard): the row's max
// key with the shard's first vocabulary row col0 folded into the index part (~(col0 + c) =
// ~c - col0: no borrow, col0 + c < 2^32), so keys of different shards compare as one row's keys;
// folded with the running key of the shards before (keys_in), stored (keys_out, may alias
// keys_in: one thread reads then writes its row) and/or decoded to the greedy id.
__global__ __launch_bounds__(1024) void argmax_keys_kernel(const unsigned long long* __restrict__ partial, int n_tiles,
                                                           unsigned int col0, const unsigned long long* keys_in,
                                                           unsigned long long* keys_out, int32_t* __restrict__ ids) {
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
    b -= (unsigned long long)col0;
    if (keys_in) {
      const unsigned long long r = keys_in[row];
      b = r > b ? r : b;
    }
    if (keys_out) keys_out[row] = b;
    if (ids) ids[row] = (int32_t)(0xFFFFFFFFu - (uint32_t)(b & 0xFFFFFFFFull));
  }
}

void launch_argmax_keys(const unsigned long long* partial, int n_tiles, int M, int col0,
                        const unsigned long long* keys_in, unsigned long long* keys_out, int32_t* ids, hipStream_t s) {
  hipLaunchKernelGGL(argmax_keys_kernel, dim3(M), dim3(1024), 0, s, partial, n_tiles, (unsigned int)col0, keys_in,
                     keys_out, ids);
}

// ids[r] from the max over n_parts shards' keys [n_parts][rows] (inferd_argmax_combine)
__global__ void argmax_combine_kernel(const unsigned long long* __restrict__ keys, int n_parts, int rows,
                                      int32_t* __restrict__ ids) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= rows) return;
  unsigned long long b = 0;
  for (int p = 0; p < n_parts; ++p) {
    const unsigned long long k = keys[(int64_t)p * rows + r];
    b = k > b ? k : b;
  }
  ids[r] = (int32_t)(0xFFFFFFFFu - (uint32_t)(b & 0xFFFFFFFFull));
}

void launch_argmax_combine(const unsigned long long* keys, int n_parts, int rows, int32_t* ids, hipStream_t s) {
  hipLaunchKernelGGL(argmax_combine_kernel, dim3((rows + 63) / 64), dim3(64), 0, s, keys, n_parts, rows, ids);
}

// ============================================================ fused prefill q/k/v projection
// launch_gemm's persistent whole-tile path with the EPI_QKV epilogue: q/k RMSNorm + RoPE to
// q_out and the K cache, V to the cache (what launch_qk_norm_rope_kv does from a stored q/k/v
// row).  Needs that path: the 4-wave persistent kernel selected, no tail split, 32-bit C offsets
// (C is unused here) and one head per wave column (N = (H + 2 KV) * 128).  The span uses it for
// every prefill; the two-kernel path (plain GEMM + qk_norm_rope) remains the reference the
// parity tests compare it with.
bool launch_gemm_qkv_fused(const u16* A, int64_t lda, const u16* Wp, int M, int N, int K, const QkvEpilogue& e,
                           hipStream_t s) {
  if (!gemm_uses_tiled(M, N, K, EPI_NONE) || !use_w4(M, N, K, EPI_NONE)) return false;
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
  const SplitTail st = {1, 0, 0, 0, nullptr, nullptr};
  hipLaunchKernelGGL(gemm_w4p_kernel<EPI_QKV>, dim3(w4p_grid(tiles)), dim3(256), 0, s, A, lda, Wp, K / 32, N / 16,
                     (u16*)nullptr, (int64_t)0, (const u16*)nullptr, (int64_t)0, M, gm, gn, st, tiles, e);
  return true;
}
