// Lab build (not product): the shipped prefill attention kernel (inferd_amd/csrc/attention.hip
// attn_prefill_kernel<3>, its page functions included from the product source unchanged) with
// per-wave s_memtime stamps around each phase, for the per-phase account of its MFMA-idle cycles
// (VERDICT r04 item 3).  tools/attn_stamps.py builds and drives it.
//
// Per wave, summed over the pages it walks (shader-clock cycles, s_memtime):
//   [0] prologue   kernel start -> q loaded and prescaled, page 0 / page 1 staging issued
//   [1] wait0      page 0's landing (the first __syncthreads)
//   [2] s_soft     S^T MFMAs + online softmax of every page (the softmax's first read of the S
//                  accumulators waits for the MFMA chain, so MFMA latency not hidden by the
//                  other wave on the SIMD lands here)
//   [3] pv         P.V + row-sum MFMAs of every page (issue; their completion is waited for by
//                  the next page's S chain or the epilogue)
//   [4] barrier    the per-page __syncthreads (next page landed, this buffer free)
//   [5] issue      the next page's LDS-DMA issue at the loop top
//   [6] epilogue   normalise + store
//   [7] pages      pages this wave computed (masked or not)
//   [8] masked     pages that ran the masked variant
//   [9] skipped    pages the wave skipped (all its rows precede them) but whose barriers it kept
//   [10] t_begin / [11] t_end  s_memrealtime (100 MHz) at kernel start / end (tail analysis)
#include "../inferd_amd/csrc/attention.hip"
#include "../include/inferd_span.h"

#define NSTAMP 12

static AttnBatch to_attn_lab(const InferdBatch* b) {
  AttnBatch a;
  a.seq_start = b->seq_start;
  a.positions = b->positions;
  a.ctx_lens = b->ctx_lens;
  a.block_table = b->block_table;
  a.max_pages = b->max_pages;
  a.B = b->n_seqs;
  a.M = b->n_tokens;
  a.max_q_len = b->max_q_len;
  a.max_ctx = b->max_ctx_len;
  return a;
}

template <int NB>
__global__ __launch_bounds__(256, 2) void attn_prefill_stamped(const u16* __restrict__ q, const u16* __restrict__ kv,
                                                            AttnBatch b, int H, int KV, float scale_log2,
                                                            u16* __restrict__ out, int order,
                                                            unsigned long long* __restrict__ stamps) {
  constexpr int QB = 64 * NB;
  constexpr int RW = 16 * NB;
  __shared__ __attribute__((aligned(16))) char lds[2 * 32768];
  const unsigned long long rt0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long acc[NSTAMP] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long tp = __builtin_amdgcn_s_memtime();
  auto lap = [&](int k) {
    const unsigned long long t = __builtin_amdgcn_s_memtime();
    acc[k] += t - tp;
    tp = t;
  };
  const int bseq = blockIdx.y;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int n_rep = H / KV;
  const int mqb = (b.max_q_len + QB - 1) / QB;
  int h, qbi;
  if (order == 1) {
    const int n = gridDim.x, x = blockIdx.x;
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
  const int qb = mqb - 1 - qbi;
  unsigned long long* rec = stamps + ((int64_t)(blockIdx.y * gridDim.x + blockIdx.x) * 4 + wave) * NSTAMP;
  if (qb >= nqb) {
    if (lane == 0) {
      for (int k = 0; k < NSTAMP; ++k) rec[k] = 0;
    }
    return;
  }
  const int qb0 = qb * QB;
  bf16x8 qf[NB][4];
  int lim[NB], tokrow[NB];
  bool valid[NB];
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
      const int piece = swave * 8 + pc;
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
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int j = 0; j < 8; ++j) qf[nb][ks][j] = (__bf16)((float)qf[nb][ks][j] * scale_log2);
  const int wg_last = b.positions[t0 + min(qb0 + QB - 1, T - 1)];
  const int wave_first_row = qb0 + wave * RW;
  const int wave_last = wave_first_row < T ? b.positions[t0 + min(wave_first_row + RW - 1, T - 1)] : -1;
  int wave_min_lim = lim[0];
#pragma unroll
  for (int nb = 1; nb < NB; ++nb) wave_min_lim = min(wave_min_lim, lim[nb]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) wave_min_lim = min(wave_min_lim, __shfl_xor(wave_min_lim, o));
  const int n_pages = wg_last / KV_PAGE + 1;
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
  if (n_pages > 1) stage(1, 1);
  lap(0);
  __syncthreads();
  lap(1);
  {
    bf16x8 pf[NB][2];
    if (KV_PAGE - 1 <= wave_min_lim) {
      prefill_page_s<false, true, NB>(lds, qf, 0, lim, m_i, ps_, o, lane, pf);
      lap(2);
      prefill_page_pv<NB>(lds + 16384, pf, o, ps_, lane);
      lap(3);
      acc[7]++;
    } else if (0 <= wave_last) {
      prefill_page_s<true, true, NB>(lds, qf, 0, lim, m_i, ps_, o, lane, pf);
      lap(2);
      prefill_page_pv<NB>(lds + 16384, pf, o, ps_, lane);
      lap(3);
      acc[7]++;
      acc[8]++;
    } else {
      acc[9]++;
    }
  }
  __syncthreads();
  lap(4);
  for (int pi = 1; pi < n_pages; ++pi) {
    const int cur = pi & 1;
    if (pi + 1 < n_pages) stage(cur ^ 1, pi + 1);
    lap(5);
    const int tok0 = pi * KV_PAGE;
    bf16x8 pf[NB][2];
    if (tok0 + KV_PAGE - 1 <= wave_min_lim) {
      prefill_page_s<false, false, NB>(lds + cur * 32768, qf, tok0, lim, m_i, ps_, o, lane, pf);
      lap(2);
      prefill_page_pv<NB>(lds + cur * 32768 + 16384, pf, o, ps_, lane);
      lap(3);
      acc[7]++;
    } else if (tok0 <= wave_last) {
      prefill_page_s<true, false, NB>(lds + cur * 32768, qf, tok0, lim, m_i, ps_, o, lane, pf);
      lap(2);
      prefill_page_pv<NB>(lds + cur * 32768 + 16384, pf, o, ps_, lane);
      lap(3);
      acc[7]++;
      acc[8]++;
    } else {
      acc[9]++;
    }
    __syncthreads();
    lap(4);
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
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  lap(6);
  acc[10] = rt0;
  acc[11] = __builtin_amdgcn_s_memrealtime();
  if (lane == 0) {  // vector stores of the wave's record
#pragma unroll
    for (int k = 0; k < NSTAMP; ++k) rec[k] = acc[k];
  }
}

extern "C" int lab_attn_prefill_stamps(const void* q, const void* kv_layer, const InferdBatch* ib, int H, int KV,
                                       void* out, void* stamps, void* stream) {
  const AttnBatch ab = to_attn_lab(ib);
  const int n = (ab.max_q_len + 191) / 192 * H;
  hipLaunchKernelGGL(attn_prefill_stamped<3>, dim3(n, ab.B), dim3(256), 0, (hipStream_t)stream, (const u16*)q,
                     (const u16*)kv_layer, ab, H, KV, 1.0f / sqrtf((float)HEAD_DIM) * LOG2E, (u16*)out,
                     n % 8 == 0 ? 1 : 0, (unsigned long long*)stamps);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

extern "C" int lab_attn_prefill_grid(const InferdBatch* ib, int H) { return (ib->max_q_len + 191) / 192 * H; }
