// GQA attention over the paged KV cache (gfx950, v_mfma_f32_16x16x32_bf16).
//
// Reference: Qwen3Attention.forward + eager_attention_forward
// (models/qwen3/server/qwen3_server_module.py:126-162, :67-89) and, for the petals span
// path, HF SDPA with the bool causal mask of petals/partitioned_models.py:28-35.
// Scores are kept in fp32 (SDPA semantics), softmax is online (flash style), P is
// rounded to bf16 for the P*V MFMA, the output is normalised in fp32 and rounded once.
//
// Both kernels compute S^T = K * Q^T (token on the MFMA row, query column on the lane)
// so that every per-query quantity (running max, sum, rescale) is lane-local and the
// S^T accumulators ARE the B operand of O^T = V^T * P^T (the V page layout in common.h
// is permuted to match).  The 16 MFMA columns are:
//   decode : the n_rep query heads that share one kv head (<= 16) of one sequence
//   prefill: 16 consecutive query rows of one head
#include "common.h"
#include "kernels.h"

#include <stdlib.h>

#define LOG2E 1.4426950408889634f

// Cross-lane helpers (gfx950 v_permlane{16,32}_swap: one VALU op, no LDS round trip).
// In the S^T accumulator layout the 4 lanes l, l^16, l^32, l^48 hold the same query.
__device__ __forceinline__ float max_q4(float v) {
  const unsigned u = __float_as_uint(v);
  auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  v = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
  const unsigned w = __float_as_uint(v);
  auto q = __builtin_amdgcn_permlane16_swap(w, w, false, false);
  return fmaxf(__uint_as_float(q[0]), __uint_as_float(q[1]));
}
__device__ __forceinline__ float sum_q4(float v) {
  const unsigned u = __float_as_uint(v);
  auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  v = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  const unsigned w = __float_as_uint(v);
  auto q = __builtin_amdgcn_permlane16_swap(w, w, false, false);
  return __uint_as_float(q[0]) + __uint_as_float(q[1]);
}
// Prefill online softmax keeps its reference max m until a row's max grows by more than
// RESCALE_THR (log2 units): p = exp2(s*c - m) <= 2^8 stays exact in fp32 and keeps bf16's
// relative precision, and the O/l rescale pass runs only on real growth (guide T13).
#define RESCALE_THR 8.0f
// bare v_exp_f32 (arguments are <= 0 or -inf here: no range reduction needed)
__device__ __forceinline__ float exp2_raw(float x) { return __builtin_amdgcn_exp2f(x); }

// ------------------------------------------------------------------ decode (1 token/seq)
// Workgroup (chunk, g, b) = NW waves over chunk `chunk` of the nc even page ranges of
// sequence b, for the n_rep query heads of kv head g; pages are interleaved over the waves
// (wave w: pages p0+w, p0+w+NW, ...).  Each wave runs a K/V software pipeline: K(i+1) is
// issued as soon as S(i) has consumed K(i), V(i+1) as soon as O += V(i) P(i) has consumed
// V(i), so one 16 KiB half-page per wave is always in flight (sched_barrier keeps the
// compiler from sinking the loads).  The NW waves merge through LDS.  A sequence with a
// single chunk writes its output directly.  Otherwise every chunk stores its unnormalised
// partial (O, m, l) and the LAST chunk to arrive merges all chunks (fixed chunk order ->
// deterministic) and resets the counter.  Hand-off per cdna_hip_programming.md §6
// Guideline 16 (write-through form): sc1 partial stores -> every wave s_waitcnt vmcnt(0) ->
// barrier -> lane 0 relaxed agent fetch_add; the last arriver: agent acquire fence +
// vmcnt(0) + barrier -> plain loads, all issued in parallel (no load inside a serial loop).
// Shape (NW, nc): the round-3 sweeps (tools/archive/attn_lab_r03.hip, archived: it includes kernels
// no longer in the tree) -- few long-running workgroups win; the launcher
// aims at ~2048 waves in total with >= 4 pages per workgroup.
// Workspace: [DECODE_COUNTER_BYTES of u32 counters | partials, PART_STRIDE f32 per head].
#define PART_STRIDE (HEAD_DIM + 4)
#define DECODE_COUNTER_BYTES 65536   // B * KV <= 16384; zero before first use, left zero
#define MAX_DECODE_CHUNKS 64

// FUSED: the kernel also does the decode token's Qwen3 QK-norm + RoPE + cache write
// (qk_norm_rope_kv_kernel's arithmetic, same rounding points): every workgroup normalises
// and rotates its n_rep query heads from the raw qkv row in registers (a lane's 32 dims of
// a head are 4 fragments; the RMS sum is reduced over the head's 4 lanes; the RoPE partner
// dim d +- 64 is the same lane's fragment ks +- 2), and the one wave that will read the
// token's page writes its K (normed, rotated) and V into the cache first, then waits for
// its own stores (vmcnt(0)) before loading that page -- no other wave reads that token.
struct DecodeFuse {
  const u16* qkv;  // bf16 [M][ldqkv] q/k/v rows, or null when `part` is given
  int64_t ldqkv;
  const u16* qn_w;
  const u16* kn_w;
  const u16* cos_t;
  const u16* sin_t;
  float eps;
  // split-K q/k/v (launch_gemm_decode_partial): value = bf16(sum_s part[s]) -- the same
  // rounding point as the unsplit GEMM's epilogue
  const float* part;  // [ksl][M][ldqkv]
  int ksl;
  // non-zero: the output is written fragment-packed (common.h packed_index) with this row
  // length (H * 128) for the o projection's decode GEMV; zero: row-major
  int64_t pack_ld;
  // decode kernel: bytes of each wave's q staging slot in dynamic LDS (0: per-lane q loads)
  int qs_bytes;
};

// q staging (fused decode attention): the workgroup's q sources -- the n_rep heads' q/k/v
// values (ksl fp32 slices, or bf16 rows), the q-norm weight and the token's cos/sin rows --
// are loaded by the wave's 64 lanes as one image (<= QS_MAXC 16-B pieces per lane) BEFORE its
// K/V ring prologue, written to the wave's LDS slot after it, and each lane then reads the
// 32 dims it needs.  vmcnt retires in order: the per-lane loads the q arithmetic used to issue
// behind the ring's 32 loads waited for all of them (probe: -2.1 us per launch without q).
constexpr int QS_MAXC = 5;  // pieces per lane: n_rep <= 4 heads x <= 2 slices (4 KiB) + 512 B
__host__ __device__ inline int q_stage_bytes(int n_rep, const float* part, int ksl) {
  return (part ? ksl * n_rep * 512 : n_rep * 256) + 512;
}

// 8 consecutive q/k/v values of row `tok` starting at column `col` (fp32, bf16-rounded)
__device__ __forceinline__ void qkv8(const DecodeFuse& f, int M, int tok, int col, float (&x)[8]) {
  if (f.part) {
    // all slices' loads issued together (predicated, unrolled to the maximum slice count)
    f32x4 pa[4], pb[4];
#pragma unroll
    for (int sl = 0; sl < 4; ++sl) {
      if (sl < f.ksl) {
        const f32x4* p = (const f32x4*)(f.part + ((int64_t)sl * M + tok) * f.ldqkv + col);
        pa[sl] = p[0];
        pb[sl] = p[1];
      } else {
        pa[sl] = pb[sl] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int sl = 0; sl < 4; ++sl) {  // fixed slice order (zeros past ksl add exactly)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[j] += pa[sl][j];
        acc[4 + j] += pb[sl][j];
      }
    }
    // the slices were normed (DN_EXACT): bf16 output of the projection
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = rbf(acc[j]);
  } else {
    const u16x8 r = *(const u16x8*)(f.qkv + (int64_t)tok * f.ldqkv + col);
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = bf2f(r[j]);
  }
}

// The Qwen3 q-norm + RoPE of one query head in the S^T fragment layout: lane l holds dims
// 8(l>>4) + 32 ks + j (ks = 0..3, j = 0..7) of query row `tok`, head `hq`; the RMS sum
// reduces over the head's 4 lanes, the RoPE partner dim d +- 64 is fragment ks +- 2 of the
// same lane.  Same per-element rounding points as qk_norm_rope_kv_kernel.
__device__ __forceinline__ void q_norm_rope_frags(const DecodeFuse& fz, int M, int tok, int pos, int hq, int lane,
                                                  bf16x8 (&qf)[4]) {
  const int d0 = 8 * (lane >> 4);
  const int qcol = hq * HEAD_DIM + d0;
  float x[4][8];
  float ss = 0.f;
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    qkv8(fz, M, tok, qcol + ks * 32, x[ks]);
#pragma unroll
    for (int j = 0; j < 8; ++j) ss += x[ks][j] * x[ks][j];
  }
  const float inv = 1.0f / sqrtf(sum_q4(ss) / 128.0f + fz.eps);
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const u16x8 wv = *(const u16x8*)(fz.qn_w + d0 + ks * 32);
#pragma unroll
    for (int j = 0; j < 8; ++j) x[ks][j] = rbf(bf2f(wv[j]) * rbf(x[ks][j] * inv));
  }
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const int dc = d0 + (ks & 1) * 32;  // dim mod 64 of element 0
    const u16x8 cv = *(const u16x8*)(fz.cos_t + (int64_t)pos * 64 + dc);
    const u16x8 sv = *(const u16x8*)(fz.sin_t + (int64_t)pos * 64 + dc);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float rot = ks < 2 ? -x[ks + 2][j] : x[ks - 2][j];
      qf[ks][j] = (__bf16)(rbf(x[ks][j] * bf2f(cv[j])) + rbf(rot * bf2f(sv[j])));
    }
  }
}

// K/V of the decode token `tok` for kv head g -> cache (lanes 0-15 K, 16-31 V; all 64 lanes
// run the arithmetic so the 16-wide shuffles see full groups)
__device__ __forceinline__ void decode_kv_write(const DecodeFuse& f, u16* __restrict__ kv, const AttnBatch& b,
                                                int bseq, int tok, int g, int H, int KV, int lane) {
  const int pos = b.positions[tok];
  const int pg = pos / KV_PAGE;
  if (pg >= b.max_pages) return;
  const int page = b.block_table[(int64_t)bseq * b.max_pages + pg], s = pos & (KV_PAGE - 1);
  const int c = lane & 15;
  float x[8];
  qkv8(f, b.M, tok, (H + g) * HEAD_DIM + c * 8, x);
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) ss += x[j] * x[j];
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 16);
  const float inv = 1.0f / sqrtf(ss / 128.0f + f.eps);
  const u16x8 wv = *(const u16x8*)(f.kn_w + c * 8);
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = rbf(bf2f(wv[j]) * rbf(x[j] * inv));
  float pr[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) pr[j] = __shfl_xor(x[j], 8, 16);
  const int ci = (c & 7) * 8;
  const u16x8 cv = *(const u16x8*)(f.cos_t + (int64_t)pos * 64 + ci);
  const u16x8 sv = *(const u16x8*)(f.sin_t + (int64_t)pos * 64 + ci);
  u16x8 ko;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float rot = c < 8 ? -pr[j] : pr[j];
    ko[j] = f2bf(rbf(x[j] * bf2f(cv[j])) + rbf(rot * bf2f(sv[j])));
  }
  if (lane < 16) {
    u16* blk = kv + kv_block(page, 0, g, KV);
    const int tb = s >> 4, ks = c >> 2, ln = (s & 15) + 16 * (c & 3);
    *(u16x8*)(blk + ((tb * 4 + ks) * 64 + ln) * 8) = ko;
  } else if (lane < 32) {
    float vx[8];
    qkv8(f, b.M, tok, (H + KV + g) * HEAD_DIM + c * 8, vx);
    u16x8 vraw;
#pragma unroll
    for (int j = 0; j < 8; ++j) vraw[j] = f2bf(vx[j]);
    u16* blk = kv + kv_block(page, 1, g, KV);
    const int kt = s >> 5, tp = s & 31;
    const int gg = tp < 16 ? (tp >> 2) : ((tp - 16) >> 2);
    const int jj = tp < 16 ? (tp & 3) : 4 + ((tp - 16) & 3);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int d = c * 8 + j;
      const int db = d >> 4, ln = (d & 15) + 16 * gg;
      blk[((kt * 8 + db) * 64 + ln) * 8 + jj] = vraw[j];
    }
  }
}

// (the ATTN_PROBE timing builds -- no q prologue / K fragments as the P*V operand -- live in
// the round-2 tree, git 6a90f3d, with tools/archive/attn_lab_r03.hip)

// Lab builds only (tools/build_probes.sh attention.hip name=-DATTN_DEC_STAMPS): per-workgroup
// s_memrealtime stamps (100 MHz) of the decode body's phases into a buffer of its own
// (inferd_lab_dec_stamps), read by tools/attn_decode_stamps.py.  Slots per workgroup:
// 0 entry, 1 q ready (wave 0), 2..9 each wave's stream end, 10 after the LDS merge barrier,
// 11 partials published (before the ticket), 12 after the ticket barrier, 13 exit, 14 flags,
// 15 the q image landed in LDS (wave 0).
#ifdef ATTN_DEC_STAMPS
#define DEC_SLOTS 16
// __constant__: the pointer comes in by a scalar load, so a stamp adds no vmcnt wait (a vector
// load of it made every stamp behind the ring prologue drain the ring)
__constant__ unsigned long long* g_dec_stamps;
__device__ __forceinline__ unsigned long long* dec_slot(int slot) {
  const unsigned wg = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  return g_dec_stamps + (size_t)wg * DEC_SLOTS + slot;
}
#define DSTAMP(slot)                                                                              \
  do {                                                                                            \
    if (threadIdx.x == 0 && g_dec_stamps) *dec_slot(slot) = __builtin_amdgcn_s_memrealtime();      \
  } while (0)
#define DSTAMP_WAVE(slot)                                                                         \
  do {                                                                                            \
    if ((threadIdx.x & 63) == 0 && g_dec_stamps)                                                  \
      *dec_slot((slot) + (threadIdx.x >> 6)) = __builtin_amdgcn_s_memrealtime();                  \
  } while (0)
#define DFLAGS(v)                                                 \
  do {                                                            \
    if (threadIdx.x == 0 && g_dec_stamps) *dec_slot(14) = (v);    \
  } while (0)
extern "C" int inferd_lab_dec_stamps(void* buf) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_dec_stamps), &buf, sizeof(buf)) == hipSuccess ? 0 : 2;
}
#else
#define DSTAMP(slot)
#define DSTAMP_WAVE(slot)
#define DFLAGS(v)
#endif

template <int NW, bool FUSED>
__device__ __forceinline__ void attn_decode_body(const u16* __restrict__ q, u16* __restrict__ kv, const AttnBatch& b,
                                                 int H, int KV, int nc_req, float scale_log2, int n_chunks_max,
                                                 unsigned* __restrict__ counters, float* __restrict__ part,
                                                 u16* __restrict__ out, const DecodeFuse& fz, const int chunk,
                                                 const int g, const int bseq) {
  __shared__ float sm_m[NW][16], sm_l[NW][16];
  __shared__ float sm_o[NW][16][HEAD_DIM + 4];
  __shared__ int sm_last;
  DSTAMP(0);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int n_rep = H / KV;
  const int ctx = b.ctx_lens[bseq];
  const int n_pages = (ctx + KV_PAGE - 1) / KV_PAGE;
  const int nc = min(nc_req, n_pages);
  if (chunk >= nc) return;
  const int cp0 = (chunk * n_pages) / nc, cp1 = ((chunk + 1) * n_pages) / nc;
  const int tok = b.seq_start[bseq + 1] - 1;
  const int hn = lane & 15;
  // Work items are 32-token half pages (K: 8 fragments, V: the 8 fragments of one kt), so
  // a chunk's 16-17 pages spread over the 8 waves in 4-5 items each instead of 2-3 pages:
  // the slowest wave sets the workgroup's time.  Halves past the last token are skipped.
  // block-table entries by scalar loads (constant address space): a vector load of the page
  // index in front of each item's addresses made every wait a vmcnt(0) that drained the ring
  typedef const __attribute__((address_space(4))) int* cptr;
  const cptr bt = (cptr)(b.block_table + (int64_t)bseq * b.max_pages);
  const int lim = ctx - 1;
  const int u_begin = 2 * cp0, u_end = min(2 * cp1, (lim >> 5) + 1);
  const int u_tok = lim >> 5;  // the token's own half page (last chunk)
  const bool writer = FUSED && chunk == nc - 1 && wave == (u_tok - u_begin) % NW;
  int u = u_begin + __builtin_amdgcn_readfirstlane(wave);  // wave-uniform: scalar block-table loads
  const bool has_item = u < u_end;
  auto kaddr = [&](int uu) {
    return (const bf16x8*)(kv + kv_block(bt[uu >> 1], 0, g, KV)) + (uu & 1) * 512 + lane;
  };
  auto vaddr = [&](int uu) {
    return (const bf16x8*)(kv + kv_block(bt[uu >> 1], 1, g, KV)) + (uu & 1) * 512 + lane;
  };
  // The first two items' K/V loads (a 2-deep register ring: item j+2 is issued as soon as
  // item j's registers are consumed, so each wave always has two half pages in flight) are
  // issued before the token's q/k/v arithmetic so their latency overlaps it.  The writer
  // stores the token's K/V first when one of those items holds the token (its stores must
  // land before it loads that half page), otherwise right after.
  bf16x8 kf[2][8], vf[2][8];
  const int u1 = u + NW;
  const bool tok_early = writer && (u == u_tok || u1 == u_tok);
  if (tok_early) {
    decode_kv_write(fz, kv, b, bseq, tok, g, H, KV, lane);
    vm_wait<0>();
  }
  // q staging: pieces c = lane + 64 i of this wave's image (unconditional loads, out-of-image
  // pieces clamped to piece 0, so the waits stay counted)
  extern __shared__ __attribute__((aligned(16))) char qs_lds[];
  const bool qstage = FUSED && fz.qs_bytes > 0;
  const int q_part_bytes = fz.part ? fz.ksl * n_rep * 512 : n_rep * 256;
  u16x8 qsr[QS_MAXC];
  if constexpr (FUSED) {
    if (qstage) {
      const int pos = lim;  // a decode token sits at its cached length (positions[tok] = ctx - 1)
#pragma unroll
      for (int i = 0; i < QS_MAXC; ++i) {
        int off = (lane + 64 * i) * 16;
        off = off < fz.qs_bytes ? off : 0;
        const char* src;
        if (off < q_part_bytes) {
          if (fz.part) {
            const int sl = off / (n_rep * 512), rem = off - sl * n_rep * 512;
            const int hh = rem >> 9, dd = (rem & 511) >> 2;
            src = (const char*)(fz.part + ((int64_t)sl * b.M + tok) * fz.ldqkv + (g * n_rep + hh) * HEAD_DIM + dd);
          } else {
            const int hh = off >> 8, e = (off & 255) >> 1;
            src = (const char*)(fz.qkv + (int64_t)tok * fz.ldqkv + (g * n_rep + hh) * HEAD_DIM + e);
          }
        } else {
          const int a = (off - q_part_bytes) >> 4;  // 0..15 q-norm weight, 16..23 cos, 24..31 sin
          src = a < 16 ? (const char*)(fz.qn_w + 8 * a)
                       : (const char*)((a < 24 ? fz.cos_t : fz.sin_t) + (int64_t)pos * 64 + 8 * ((a - 16) & 7));
        }
        qsr[i] = *(const u16x8*)src;
      }
    }
  }
  auto load_item = [&](auto ST, int uu) {
    constexpr int st = decltype(ST)::value;
    const bf16x8* kb = kaddr(uu);
    const bf16x8* vb = vaddr(uu);
#pragma unroll
    for (int i = 0; i < 8; ++i) kf[st][i] = __builtin_nontemporal_load(kb + i * 64);
#pragma unroll
    for (int i = 0; i < 8; ++i) vf[st][i] = __builtin_nontemporal_load(vb + i * 64);
  };
  // both stages unconditionally (a wave with one item loads it twice, a wave with none loads
  // the chunk's first item): an issue guarded by a branch makes hipcc's waitcnt pass merge
  // the paths and drain the ring (vmcnt(0))
  load_item(std::integral_constant<int, 0>{}, has_item ? u : u_begin);
  load_item(std::integral_constant<int, 1>{}, u1 < u_end ? u1 : (has_item ? u : u_begin));
  bf16x8 qf[4];
  if constexpr (FUSED) {
    const int hh = hn < n_rep ? hn : 0;
    if (qstage) {
      char* qs = qs_lds + wave * fz.qs_bytes;
#pragma unroll
      for (int i = 0; i < QS_MAXC; ++i)
        if ((lane + 64 * i) * 16 < fz.qs_bytes) *(u16x8*)(qs + (lane + 64 * i) * 16) = qsr[i];
      DSTAMP(15);
      // this wave's own LDS slot: its stores are read back by its own lanes only
      const int d0 = 8 * (lane >> 4);
      float x[4][8];
      float ss = 0.f;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        if (fz.part) {
          const float* p0 = (const float*)(qs + hh * 512) + d0 + ks * 32;
          f32x4 a0 = *(const f32x4*)p0, a1 = *(const f32x4*)(p0 + 4), b0 = a0 * 0.f, b1 = a1 * 0.f;
          if (fz.ksl == 2) {
            const float* p1 = (const float*)(qs + (n_rep + hh) * 512) + d0 + ks * 32;
            b0 = *(const f32x4*)p1;
            b1 = *(const f32x4*)(p1 + 4);
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) {  // slice order as qkv8: 0 + s0 + s1
            x[ks][j] = rbf(0.f + a0[j] + b0[j]);
            x[ks][4 + j] = rbf(0.f + a1[j] + b1[j]);
          }
        } else {
          const u16x8 r = *(const u16x8*)(qs + hh * 256 + (d0 + ks * 32) * 2);
#pragma unroll
          for (int j = 0; j < 8; ++j) x[ks][j] = bf2f(r[j]);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) ss += x[ks][j] * x[ks][j];
      }
      const float inv = 1.0f / sqrtf(sum_q4(ss) / 128.0f + fz.eps);
      const u16* aux = (const u16*)(qs + q_part_bytes);
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const u16x8 wv = *(const u16x8*)(aux + d0 + ks * 32);
#pragma unroll
        for (int j = 0; j < 8; ++j) x[ks][j] = rbf(bf2f(wv[j]) * rbf(x[ks][j] * inv));
      }
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int dc = d0 + (ks & 1) * 32;
        const u16x8 cv = *(const u16x8*)(aux + 128 + dc);
        const u16x8 sv = *(const u16x8*)(aux + 192 + dc);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float rot = ks < 2 ? -x[ks + 2][j] : x[ks - 2][j];
          qf[ks][j] = (__bf16)(rbf(x[ks][j] * bf2f(cv[j])) + rbf(rot * bf2f(sv[j])));
        }
      }
    } else {
      q_norm_rope_frags(fz, b.M, tok, b.positions[tok], g * n_rep + hh, lane, qf);
    }
  } else {
    const int hh = hn < n_rep ? hn : 0;
    const u16* qp = q + ((int64_t)tok * H + g * n_rep + hh) * HEAD_DIM + 8 * (lane >> 4);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) qf[ks] = *(const bf16x8*)(qp + ks * 32);
  }
  // the writer's token K/V when none of its first two items holds the token: its stores land
  // before the ring refills with the token's half page (item(): vm_wait before that issue)
  if (writer && !tok_early) decode_kv_write(fz, kv, b, bseq, tok, g, H, KV, lane);
  DSTAMP(1);
  float m_i = -INFINITY, l_i = 0.f;
  f32x4 o[8];
#pragma unroll
  for (int db = 0; db < 8; ++db) o[db] = f32x4{0.f, 0.f, 0.f, 0.f};
  // one item with its registers in ring stage ST; ISSUE: refill the stage with item u + 2 NW
  // (the caller knows statically whether it exists -- see the loop below)
  auto item = [&](auto ST, auto ISSUE) {
    constexpr int st = decltype(ST)::value;
    constexpr bool more = decltype(ISSUE)::value;
    const int nxt = u + 2 * NW;  // refills this stage
    const int tok0 = u * 32;
    f32x4 sc[2];
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2) {
      sc[t2] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) sc[t2] = mfma16(kf[st][t2 * 4 + ks], qf[ks], sc[t2]);
    }
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (more) {
      if (writer && nxt == u_tok) vm_wait<0>();
      const bf16x8* kb = kaddr(nxt);
#pragma unroll
      for (int i = 0; i < 8; ++i) kf[st][i] = __builtin_nontemporal_load(kb + i * 64);
    }
    __builtin_amdgcn_sched_barrier(0);
    if (tok0 + 31 > lim) {  // the half page holding the token: length mask
#pragma unroll
      for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int t = tok0 + t2 * 16 + 4 * (lane >> 4) + r;
          sc[t2][r] = (t <= lim) ? sc[t2][r] : -INFINITY;
        }
    }
    const float pmax = fmaxf(fmaxf(fmaxf(sc[0][0], sc[0][1]), fmaxf(sc[0][2], sc[0][3])),
                             fmaxf(fmaxf(sc[1][0], sc[1][1]), fmaxf(sc[1][2], sc[1][3])));
    const float m_new = fmaxf(m_i, max_q4(pmax) * scale_log2);
    if (__builtin_amdgcn_ballot_w64(m_new > m_i)) {
      const float alpha = exp2_raw(m_i - m_new);
      l_i *= alpha;
#pragma unroll
      for (int db = 0; db < 8; ++db) o[db] *= alpha;
      m_i = m_new;
    }
    const float mneg = -m_i;
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
      for (int r = 0; r < 4; ++r) sc[t2][r] = exp2_raw(fmaf(sc[t2][r], scale_log2, mneg));
    // this lane's share of the row sum; reduced over the query's 4 lanes after the loop
    l_i += ((sc[0][0] + sc[0][1]) + (sc[0][2] + sc[0][3])) + ((sc[1][0] + sc[1][1]) + (sc[1][2] + sc[1][3]));
    bf16x8 pf;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      pf[j] = (__bf16)sc[0][j];
      pf[4 + j] = (__bf16)sc[1][j];
    }
#pragma unroll
    for (int db = 0; db < 8; ++db) o[db] = mfma16(vf[st][db], pf, o[db]);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (more) {
      const bf16x8* vb = vaddr(nxt);
#pragma unroll
      for (int i = 0; i < 8; ++i) vf[st][i] = __builtin_nontemporal_load(vb + i * 64);
    }
    __builtin_amdgcn_sched_barrier(0);
    u += NW;
  };
  if (has_item) {
    using S0 = std::integral_constant<int, 0>;
    using S1 = std::integral_constant<int, 1>;
    using Y = std::true_type;
    using N = std::false_type;
    // steady state: both items of a pass refill their stage; then 1-3 items remain, run as
    // straight-line tails (no guarded loads anywhere, so every wait is counted exactly)
    while (u + 3 * NW < u_end) {
      item(S0{}, Y{});
      item(S1{}, Y{});
    }
    const int rem = (u_end - u + NW - 1) / NW;
    if (rem == 3) {
      item(S0{}, Y{});
      item(S1{}, N{});
      item(S0{}, N{});
    } else if (rem == 2) {
      item(S0{}, N{});
      item(S1{}, N{});
    } else {
      item(S0{}, N{});
    }
  }
  DSTAMP_WAVE(2);
  // merge the NW waves through LDS
  l_i = sum_q4(l_i);
  if (lane < 16) {
    sm_m[wave][lane] = m_i;
    sm_l[wave][lane] = l_i;
  }
#pragma unroll
  for (int db = 0; db < 8; ++db)
#pragma unroll
    for (int r = 0; r < 4; ++r) sm_o[wave][hn][db * 16 + 4 * (lane >> 4) + r] = o[db][r];
  __syncthreads();
  DSTAMP(10);
  u16* op = out + (int64_t)tok * H * HEAD_DIM + (int64_t)g * n_rep * HEAD_DIM;
  const int stride = n_rep * PART_STRIDE;
  float* base = part + ((int64_t)bseq * KV + g) * n_chunks_max * stride;
  for (int idx = threadIdx.x; idx < n_rep * HEAD_DIM; idx += NW * 64) {
    const int n = idx / HEAD_DIM, d = idx % HEAD_DIM;
    float M = sm_m[0][n];
#pragma unroll
    for (int w = 1; w < NW; ++w) M = fmaxf(M, sm_m[w][n]);
    float acc = 0.f, L = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const float f = (sm_m[w][n] == -INFINITY) ? 0.f : exp2f(sm_m[w][n] - M);
      acc += sm_o[w][n][d] * f;
      L += sm_l[w][n] * f;
    }
    if (nc == 1) {
      const u16 ov = f2bf(acc / L);
      if (fz.pack_ld) out[packed_index(tok, (g * n_rep + n) * HEAD_DIM + d, fz.pack_ld)] = ov;
      else op[n * HEAD_DIM + d] = ov;
    } else {
      float* pc = base + (int64_t)chunk * stride + n * PART_STRIDE;
      __hip_atomic_store(pc + d, acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (d == 0) {
        __hip_atomic_store(pc + HEAD_DIM, M, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(pc + HEAD_DIM + 1, L, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  if (nc == 1) {
    DSTAMP(13);
    DFLAGS(1ull | ((unsigned long long)nc << 8) | ((unsigned long long)chunk << 16));
    return;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  DSTAMP(11);
  if (threadIdx.x == 0) {
    const unsigned prev =
        __hip_atomic_fetch_add(&counters[bseq * KV + g], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    sm_last = (prev == (unsigned)(nc - 1));
    if (sm_last) __hip_atomic_store(&counters[bseq * KV + g], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  DSTAMP(12);
  DFLAGS((unsigned long long)sm_last | ((unsigned long long)nc << 8) | ((unsigned long long)chunk << 16));
  if (!sm_last) {
    DSTAMP(13);
    return;
  }
  // Last arriver: every partial was stored write-through (sc1) and drained before its
  // workgroup's ticket add, and every load of one here is an sc1 load, so no acquire fence
  // is needed (MI355X_MICROARCH.md, visibility "Valid forms", row 1: one workgroup per CU,
  // unsharded counter, last adder told by the returned value).  One pass per (head, dim),
  // chunks merged in fixed order (deterministic).  The chunks' (m, l, o) are loaded MB at a
  // time from clamped addresses, all issued before the first use: one memory round trip per
  // MB chunks (a loop of dependent loads cost two round trips per chunk: nc = 16 took 118 us).
  constexpr int MB = 8;
  auto ld = [](const float* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  for (int idx = threadIdx.x; idx < n_rep * HEAD_DIM; idx += NW * 64) {
    const int n = idx / HEAD_DIM, d = idx % HEAD_DIM;
    const float* pn = base + n * PART_STRIDE;
    float mc[MB], lc[MB], oc[MB];
    auto load_block = [&](int c0) {
#pragma unroll
      for (int j = 0; j < MB; ++j) {
        const float* pc = pn + (int64_t)min(c0 + j, nc - 1) * stride;
        mc[j] = ld(pc + HEAD_DIM);
        lc[j] = ld(pc + HEAD_DIM + 1);
        oc[j] = ld(pc + d);
      }
    };
    load_block(0);
    float M = -INFINITY;
    for (int c0 = 0; c0 < nc; c0 += MB) {
      if (c0) load_block(c0);
#pragma unroll
      for (int j = 0; j < MB; ++j)
        if (c0 + j < nc) M = fmaxf(M, mc[j]);
    }
    if (nc > MB) load_block(0);
    float acc = 0.f, L = 0.f;
    for (int c0 = 0; c0 < nc; c0 += MB) {
      if (c0) load_block(c0);
#pragma unroll
      for (int j = 0; j < MB; ++j)
        if (c0 + j < nc) {
          const float f = exp2f(mc[j] - M);
          L += lc[j] * f;
          acc += oc[j] * f;
        }
    }
    const u16 ov = f2bf(acc / L);
    if (fz.pack_ld) out[packed_index(tok, (g * n_rep + n) * HEAD_DIM + d, fz.pack_ld)] = ov;
    else op[n * HEAD_DIM + d] = ov;
  }
#ifdef ATTN_DEC_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
#endif
  DSTAMP(13);
}

template <int NW, bool FUSED>
__global__ __launch_bounds__(NW * 64) void attn_decode_kernel(const u16* __restrict__ q, u16* __restrict__ kv,
                                                      AttnBatch b, int H, int KV, int nc_req, float scale_log2,
                                                      int n_chunks_max, unsigned* __restrict__ counters,
                                                      float* __restrict__ part, u16* __restrict__ out,
                                                      DecodeFuse fz) {
  attn_decode_body<NW, FUSED>(q, kv, b, H, KV, nc_req, scale_log2, n_chunks_max, counters, part, out, fz,
                              blockIdx.x, blockIdx.y, blockIdx.z);
}

// (waves per workgroup, chunks per (seq, kv head)) for a decode batch (the round-3 shape sweep measured
// the alternatives with lab builds)
static void decode_shape(int B, int KV, int max_ctx, int* nw, int* nc) {
  const int np = (max_ctx + KV_PAGE - 1) / KV_PAGE;
  const int S = B * KV;
  const int w = (S * 8 <= 2048 && np < 96) ? 8 : 4;
  int c = 2048 / (S * w);
  const int cmax = np / 4 > 1 ? np / 4 : 1;
  c = c < 1 ? 1 : (c > cmax ? cmax : c);
  if (c > MAX_DECODE_CHUNKS) c = MAX_DECODE_CHUNKS;
  *nw = w;
  *nc = c;
}

size_t attn_decode_ws_bytes(int B, int H, int max_ctx) {
  // worst case over kv-head counts (KV <= H): MAX_DECODE_CHUNKS chunks of n_rep heads
  return DECODE_COUNTER_BYTES + (size_t)B * H * MAX_DECODE_CHUNKS * PART_STRIDE * sizeof(float);
}

template <bool FUSED>
static void attn_decode_go(const u16* q, u16* kv_layer, const AttnBatch& b, int H, int KV, float scale, u16* out,
                           float* ws, hipStream_t s, const DecodeFuse& fz_in) {
  int nw, nc;
  decode_shape(b.B, KV, b.max_ctx, &nw, &nc);
  unsigned* counters = (unsigned*)ws;
  float* part = (float*)((char*)ws + DECODE_COUNTER_BYTES);
  DecodeFuse fz = fz_in;
  const int n_rep = H / KV;
  const int qsb = q_stage_bytes(n_rep, fz.part, fz.ksl);
  fz.qs_bytes = (FUSED && n_rep <= 4 && (!fz.part || fz.ksl <= 2) && qsb <= QS_MAXC * 1024)
                    ? qsb
                    : 0;
  const unsigned lds = (unsigned)(nw * fz.qs_bytes);
  if (nw == 8)
    hipLaunchKernelGGL((attn_decode_kernel<8, FUSED>), dim3(nc, KV, b.B), dim3(512), lds, s, q, kv_layer, b, H, KV,
                       nc, scale * LOG2E, nc, counters, part, out, fz);
  else
    hipLaunchKernelGGL((attn_decode_kernel<4, FUSED>), dim3(nc, KV, b.B), dim3(256), lds, s, q, kv_layer, b, H, KV,
                       nc, scale * LOG2E, nc, counters, part, out, fz);
}

void launch_attn_decode(const u16* q, const u16* kv_layer, const AttnBatch& b, int H, int KV,
                        float scale, u16* out, float* ws, hipStream_t s) {
  attn_decode_go<false>(q, (u16*)kv_layer, b, H, KV, scale, out, ws, s, DecodeFuse{});
}

void launch_attn_decode_fused(const u16* qkv, int64_t ldqkv, const u16* qn_w, const u16* kn_w, const u16* cos_t,
                              const u16* sin_t, float eps, u16* kv_layer, const AttnBatch& b, int H, int KV,
                              float scale, u16* out, float* ws, hipStream_t s, const float* part, int ksl,
                              bool pack_out) {
  const DecodeFuse fz = {qkv, ldqkv, qn_w, kn_w, cos_t, sin_t, eps, part, ksl, pack_out ? (int64_t)H * HEAD_DIM : 0};
  attn_decode_go<true>(nullptr, kv_layer, b, H, KV, scale, out, ws, s, fz);
}

// ------------------------------------------------------------------ prefill (causal)
// grid (ceil(max_q_len/(64 NB)), H, B), 4 waves.  The workgroup owns 64 NB query rows of one head
// (NB = 3 by default: 192); wave w owns 16 NB rows as NB 16-row MFMA column blocks.  Every K/V page (K 16 KiB
// + V 16 KiB of this kv head) is staged ONCE per workgroup into double-buffered LDS with
// global_load_lds_dwordx4 (32 x 1 KiB pieces, 8 per wave) while the previous page is being
// consumed; the page layout is already fragment-ordered, so every fragment read is
// lds[tile * 1 KiB + lane * 16] (contiguous, bank-conflict free), and each K/V fragment feeds
// the MFMAs of all NB column blocks.  Waves whose rows all precede a page skip its compute but
// keep the barriers.
//
// Softmax VALU per page was the kernel's pole (64 MFMAs vs ~550 VALU ops in round 1), so:
//  * the causal mask is applied only on pages that cross one of the wave's rows' limits
//    (wave-uniform test), every other page is mask-free;
//  * the scale is folded into Q (q' = bf16(q * scale * log2 e), once per workgroup) and the
//    running reference max -m rides the first S MFMA's C operand, so the accumulators come out as
//    s' = q'.k - m and p = exp2(s') is one bare v_exp_f32 per score (arguments <= 0 / -inf save
//    the lazy-rescale slack), no fma;
//  * the row sum l comes out of the P.V MFMAs: one more 16x16x32 MFMA per 32 tokens against an
//    all-ones A operand gives sum_t bf16(p_t) -- the sum of exactly the weights P.V uses -- in
//    every lane of the query, with no VALU add and no cross-lane reduction;
//  * the first page (token 0, visible to every row) sets m exactly; afterwards a row's max moves
//    only when it grows by more than RESCALE_THR (wave-uniform branch), and then o, l and this
//    page's s' shift by the growth (guide T13: nothing at the old max is left unscaled);
//  * row max reductions use v_permlane{32,16}_swap instead of ds_bpermute.
// The two rounding moves (q rounded as bf16(q * c) instead of bf16(q); l the sum of bf16 p) were
// measured on the 32B / 8k shape (tools/attn_ab.py, profiles/r04/attn_ab.txt): 1019.6 -> 944.2 us,
// rms error against fp32 attention 2.13e-3 -> 2.75e-3; the config-5 noise-floor test
// (test_config5_q32b_layer_prefill_8192) holds the layer to the bf16 reference's distance from fp32.
struct PfState {
  f32x4 negm;  // (-m) x 4: the S chains' initial C operand
  f32x4 l;     // row sum (every element the same)
};
// S^T of a page (K at kl) + its online softmax -> P (bf16, the B operand of P.V) in pf
template <bool MASK, bool FIRST, int NB>
__device__ __forceinline__ void prefill_page_s(const char* __restrict__ kl, const bf16x8 (&qf)[NB][4], int page_tok0,
                                               const int (&lim)[NB], float (&m_i)[NB], PfState (&ps_)[NB],
                                               f32x4 (&o)[NB][8], int lane, bf16x8 (&pf)[NB][2]) {
  const char* lds = kl;
  f32x4 sc[NB][4];
  // k-slice outermost: eight accumulation chains in flight (tb outermost left two, with
  // s_nops between dependent MFMAs)
#pragma unroll
  for (int ks = 0; ks < 4; ++ks)
#pragma unroll
    for (int tb = 0; tb < 4; ++tb) {
      const bf16x8 kf = *(const bf16x8*)(lds + (tb * 4 + ks) * 1024 + lane * 16);
#pragma unroll
      for (int nb = 0; nb < NB; ++nb)
        sc[nb][tb] = mfma16(kf, qf[nb][ks], ks ? sc[nb][tb] : (FIRST ? f32x4{0.f, 0.f, 0.f, 0.f} : ps_[nb].negm));
    }
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    if constexpr (MASK) {
#pragma unroll
      for (int tb = 0; tb < 4; ++tb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int t = page_tok0 + tb * 16 + 4 * (lane >> 4) + r;
          sc[nb][tb][r] = (t <= lim[nb]) ? sc[nb][tb][r] : -INFINITY;
        }
    }
    float pm[4];  // 4 independent max chains
#pragma unroll
    for (int tb = 0; tb < 4; ++tb)
      pm[tb] = fmaxf(fmaxf(sc[nb][tb][0], sc[nb][tb][1]), fmaxf(sc[nb][tb][2], sc[nb][tb][3]));
    const float pmax = max_q4(fmaxf(fmaxf(pm[0], pm[1]), fmaxf(pm[2], pm[3])));
    // sc = s' = s c - m (m = 0 on the first page)
    float shift = 0.f;
    if constexpr (FIRST) {
      shift = pmax;  // finite: token 0 is visible to every row
      m_i[nb] = pmax;
      ps_[nb].negm = f32x4{-pmax, -pmax, -pmax, -pmax};
    } else if (__builtin_amdgcn_ballot_w64(pmax > RESCALE_THR)) {
      shift = fmaxf(pmax, 0.f);  // -inf (all masked) -> no shift
      const float alpha = exp2_raw(-shift);
      ps_[nb].l *= alpha;
#pragma unroll
      for (int db = 0; db < 8; ++db) o[nb][db] *= alpha;
      m_i[nb] += shift;
      ps_[nb].negm = f32x4{-m_i[nb], -m_i[nb], -m_i[nb], -m_i[nb]};
    }
    if (FIRST || shift != 0.f) {
#pragma unroll
      for (int tb = 0; tb < 4; ++tb) sc[nb][tb] -= shift;
    }
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pf[nb][kt][j] = (__bf16)exp2_raw(sc[nb][2 * kt][j]);
        pf[nb][kt][4 + j] = (__bf16)exp2_raw(sc[nb][2 * kt + 1][j]);
      }
  }
}
// O^T += V^T P^T of a page (V at vl), and l += 1^T P^T on the same P operands
template <int NB>
__device__ __forceinline__ void prefill_page_pv(const char* __restrict__ vl, const bf16x8 (&pf)[NB][2],
                                                f32x4 (&o)[NB][8], PfState (&ps_)[NB], int lane) {
  bf16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (__bf16)1.0f;
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
    for (int db = 0; db < 8; ++db) {
      const bf16x8 vf = *(const bf16x8*)(vl + (kt * 8 + db) * 1024 + lane * 16);
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) o[nb][db] = mfma16(vf, pf[nb][kt], o[nb][db]);
    }
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) ps_[nb].l = mfma16(ones, pf[nb][kt], ps_[nb].l);
  }
}
template <bool MASK, bool FIRST, int NB>
__device__ __forceinline__ void prefill_page_lds(const char* __restrict__ lds, const bf16x8 (&qf)[NB][4],
                                                 int page_tok0, const int (&lim)[NB], float (&m_i)[NB],
                                                 PfState (&ps_)[NB], f32x4 (&o)[NB][8], int lane) {
  bf16x8 pf[NB][2];
  prefill_page_s<MASK, FIRST, NB>(lds, qf, page_tok0, lim, m_i, ps_, o, lane, pf);
  prefill_page_pv<NB>(lds + 16384, pf, o, ps_, lane);
}

// Block order (grid x = max_q_blocks * H per sequence, y = sequence): mode 1 (used when
// that count is a multiple of 8) deals each XCD a contiguous range of (kv group, query block,
// head) with the n_rep heads of a group fastest, so the heads that read the same K/V pages
// run together on one XCD (one L2); query blocks heaviest first, so light blocks fill the
// tail.  Mode 0: head-major, heaviest query block first.
// NB: 16-row MFMA column blocks per wave (each staged K/V fragment feeds NB MFMAs): 3 = 192 rows
// per workgroup (a third fewer LDS fragment reads per MFMA than 2 = 128 rows; 256 VGPRs with
// a few bytes of scratch, measured faster anyway: 944 vs 994 us at 32B / 8k with the cuts)
template <int NB>
__global__ __launch_bounds__(256, 2) void attn_prefill_kernel(const u16* __restrict__ q,
                                                           const u16* __restrict__ kv,
                                                           AttnBatch b, int H, int KV,
                                                           float scale_log2,
                                                           u16* __restrict__ out, int order) {
  constexpr int QB = 64 * NB;  // query rows per workgroup
  constexpr int RW = 16 * NB;  // per wave
  __shared__ __attribute__((aligned(16))) char lds[2 * 32768];
  const int bseq = blockIdx.y;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int n_rep = H / KV;
  const int mqb = (b.max_q_len + QB - 1) / QB;  // query blocks per head in the grid
  int h, qbi;
  if (order == 1) {
    const int n = gridDim.x, x = blockIdx.x;  // n % 8 == 0 (launcher)
    const int wg = (x & 7) * (n >> 3) + (x >> 3);
    const int r = wg % n_rep, t = wg / n_rep;
    qbi = t % mqb;
    h = (t / mqb) * n_rep + r;
  } else {
    h = blockIdx.x / mqb;
    qbi = blockIdx.x % mqb;
  }
  const int g = h / n_rep;
  const int t0 = b.seq_start[bseq];
  const int T = b.seq_start[bseq + 1] - t0;
  const int nqb = (T + QB - 1) / QB;
  // heaviest (latest) query blocks first
  const int qb = mqb - 1 - qbi;
  if (qb >= nqb) return;  // uniform over the workgroup
  const int qb0 = qb * QB;
  bf16x8 qf[NB][4];
  int lim[NB], tokrow[NB];
  bool valid[NB];
  // page 0's K/V go in flight first: the q loads and their prescale below then overlap its
  // latency instead of preceding it (one round trip per workgroup instead of two)
  typedef const __attribute__((address_space(4))) int* cptr;
  typedef __attribute__((address_space(3))) void* lds_ptr;
  const cptr bt = (cptr)(b.block_table + (int64_t)bseq * b.max_pages);
  const int swave = __builtin_amdgcn_readfirstlane(wave);
  auto stage = [&](int buf, int pi) {
    const __amdgpu_buffer_rsrc_t pg_rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void*)(kv + kv_block(bt[pi], 0, g, KV)), 0, 2 * KV_BLOCK_ELEMS * 2, 0x00020000);
    char* base = lds + buf * 32768;
#pragma unroll
    for (int pc = 0; pc < 8; ++pc) {
      const int piece = swave * 8 + pc;  // 0..15 K tiles, 16..31 V tiles
      __builtin_amdgcn_raw_ptr_buffer_load_lds(pg_rsrc, (lds_ptr)(base + piece * 1024), 16, lane * 16, piece * 1024, 0,
                                               0);
    }
  };
  stage(0, 0);
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    const int row = qb0 + wave * RW + nb * 16 + (lane & 15);
    valid[nb] = row < T;
    tokrow[nb] = t0 + (valid[nb] ? row : T - 1);
    lim[nb] = b.positions[tokrow[nb]];
    const u16* qp = q + ((int64_t)tokrow[nb] * H + h) * HEAD_DIM + 8 * (lane >> 4);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) qf[nb][ks] = *(const bf16x8*)(qp + ks * 32);
  }
  // q' = bf16(q * scale * log2 e)
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int j = 0; j < 8; ++j) qf[nb][ks][j] = (__bf16)((float)qf[nb][ks][j] * scale_log2);
  // pages: up to the workgroup's last row; a wave computes up to its own last row and
  // masks only pages that reach past its smallest row limit
  const int wg_last = b.positions[t0 + min(qb0 + QB - 1, T - 1)];
  const int wave_first_row = qb0 + wave * RW;
  const int wave_last = wave_first_row < T ? b.positions[t0 + min(wave_first_row + RW - 1, T - 1)] : -1;
  int wave_min_lim = lim[0];
#pragma unroll
  for (int nb = 1; nb < NB; ++nb) wave_min_lim = min(wave_min_lim, lim[nb]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) wave_min_lim = min(wave_min_lim, __shfl_xor(wave_min_lim, o));
  const int n_pages = wg_last / KV_PAGE + 1;
  // (K/V staging, `stage` above: buffer_load ... lds with one wave-uniform descriptor per page --
  // its 64-bit base from a scalar load of the block table, in SGPRs -- the piece offsets in
  // SGPRs, lane * 16 the only VGPR; the per-piece 64-bit address arithmetic of global_load_lds
  // was ~60 VALU per page per wave.  A page's K block is followed by its V block (common.h
  // kv_block), so its 32 pieces are one contiguous 32 KiB run: the descriptor covers exactly
  // that run, whatever the pool size.)
  float m_i[NB];
  PfState ps_[NB];
  f32x4 o[NB][8];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    m_i[nb] = -INFINITY;
    ps_[nb].negm = f32x4{0.f, 0.f, 0.f, 0.f};
    ps_[nb].l = f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int db = 0; db < 8; ++db) o[nb][db] = f32x4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();
  // page 0 (token 0: every row's first visible key) sets the rows' reference max
  if (n_pages > 1) stage(1, 1);
  if (KV_PAGE - 1 <= wave_min_lim)
    prefill_page_lds<false, true, NB>(lds, qf, 0, lim, m_i, ps_, o, lane);
  else if (0 <= wave_last)
    prefill_page_lds<true, true, NB>(lds, qf, 0, lim, m_i, ps_, o, lane);
  __syncthreads();
  for (int pi = 1; pi < n_pages; ++pi) {
    const int cur = pi & 1;
    if (pi + 1 < n_pages) stage(cur ^ 1, pi + 1);
    const int tok0 = pi * KV_PAGE;
    if (tok0 + KV_PAGE - 1 <= wave_min_lim)
      prefill_page_lds<false, false, NB>(lds + cur * 32768, qf, tok0, lim, m_i, ps_, o, lane);
    else if (tok0 <= wave_last)
      prefill_page_lds<true, false, NB>(lds + cur * 32768, qf, tok0, lim, m_i, ps_, o, lane);
    __syncthreads();  // next page landed (vmcnt(0)) and everyone is done with this buffer
  }
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    const float inv = 1.0f / ps_[nb].l[0];
    if (!valid[nb]) continue;
    u16* op = out + (int64_t)tokrow[nb] * H * HEAD_DIM + h * HEAD_DIM;
#pragma unroll
    for (int db = 0; db < 8; ++db) {
      u16x4 v;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = f2bf(o[nb][db][r] * inv);
      *(u16x4*)(op + db * 16 + 4 * (lane >> 4)) = v;
    }
  }
}

#ifdef ATTN_W64
// lab builds only (tools/build_w64_lab.sh): the one-wave-per-SIMD body of tools/labsrc/attn_w64.hip
bool launch_attn_prefill_w64(const u16* q, const u16* kv_layer, const AttnBatch& b, int H, int KV, float scale,
                             u16* out, hipStream_t s);
#endif
void launch_attn_prefill(const u16* q, const u16* kv_layer, const AttnBatch& b, int H, int KV, float scale, u16* out,
                         hipStream_t s) {
#ifdef ATTN_W64
  if (launch_attn_prefill_w64(q, kv_layer, b, H, KV, scale, out, s)) return;
#endif
  // 48 query rows per wave; XCD-grouped block order whenever the grid allows it
  const int n = (b.max_q_len + 191) / 192 * H;
  hipLaunchKernelGGL(attn_prefill_kernel<3>, dim3(n, b.B), dim3(256), 0, s, q, kv_layer, b, H, KV, scale * LOG2E, out,
                     n % 8 == 0 ? 1 : 0);
}
