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

// One 64-token page of online-softmax attention for one wave.
// qf: Q^T fragments (4 k-steps of 32 dims); keys t <= lim are visible (lane-local limit).
__device__ __forceinline__ void attend_page(const u16* __restrict__ kblk, const u16* __restrict__ vblk,
                                            const bf16x8 (&qf)[4], int page_tok0, int lim,
                                            float scale_log2, float& m_i, float& l_i,
                                            f32x4 (&o)[8], int lane) {
  const bf16x8* kb = (const bf16x8*)kblk + lane;
  const bf16x8* vb = (const bf16x8*)vblk + lane;
  bf16x8 kf[16], vf[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) kf[i] = kb[i * 64];
#pragma unroll
  for (int i = 0; i < 16; ++i) vf[i] = vb[i * 64];
  f32x4 sc[4];
#pragma unroll
  for (int tb = 0; tb < 4; ++tb) {
    sc[tb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) sc[tb] = mfma16(kf[tb * 4 + ks], qf[ks], sc[tb]);
  }
  float pmax = -INFINITY;
#pragma unroll
  for (int tb = 0; tb < 4; ++tb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int t = page_tok0 + tb * 16 + 4 * (lane >> 4) + r;
      const float s = (t <= lim) ? sc[tb][r] * scale_log2 : -INFINITY;
      sc[tb][r] = s;
      pmax = fmaxf(pmax, s);
    }
  pmax = fmaxf(pmax, __shfl_xor(pmax, 16));
  pmax = fmaxf(pmax, __shfl_xor(pmax, 32));
  const float m_new = fmaxf(m_i, pmax);
  const float alpha = exp2f(m_i - m_new);
  float psum = 0.f;
#pragma unroll
  for (int tb = 0; tb < 4; ++tb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float p = exp2f(sc[tb][r] - m_new);
      sc[tb][r] = p;
      psum += p;
    }
  psum += __shfl_xor(psum, 16);
  psum += __shfl_xor(psum, 32);
  l_i = l_i * alpha + psum;
  m_i = m_new;
#pragma unroll
  for (int db = 0; db < 8; ++db) o[db] *= alpha;
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
    bf16x8 pf;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      pf[j] = (__bf16)sc[2 * kt][j];
      pf[4 + j] = (__bf16)sc[2 * kt + 1][j];
    }
#pragma unroll
    for (int db = 0; db < 8; ++db) o[db] = mfma16(vf[kt * 8 + db], pf, o[db]);
  }
}

// ------------------------------------------------------------------ decode (1 token/seq)
// Workgroup (chunk, g, b) = 4 waves; wave w attends pages [chunk*4*ppw + w*ppw, +ppw) of
// sequence b for the n_rep query heads of kv head g; the 4 waves merge through LDS.  A
// sequence with a single chunk writes its output directly.  Otherwise every chunk stores
// its unnormalised partial (O, m, l) and the LAST chunk to arrive merges all chunks
// (fixed chunk order -> deterministic) and resets the counter.  Hand-off per
// cdna_hip_programming.md §6 Guideline 16 (write-through form): sc1 partial stores -> every
// wave s_waitcnt vmcnt(0) -> barrier -> lane 0 relaxed agent fetch_add; the last arriver:
// agent acquire fence + vmcnt(0) + barrier -> plain loads.
// The merge is parallel: per-chunk scale factors first (LDS), then independent loads.
// Workspace: [DECODE_COUNTER_BYTES of u32 counters | partials, PART_STRIDE f32 per head].
#define PART_STRIDE (HEAD_DIM + 4)
#define DECODE_COUNTER_BYTES 65536   // B * KV <= 16384; zero before first use, left zero
#define MAX_DECODE_CHUNKS 64

__global__ __launch_bounds__(256) void attn_decode_kernel(const u16* __restrict__ q,
                                                          const u16* __restrict__ kv, AttnBatch b,
                                                          int H, int KV, int ppw, float scale_log2,
                                                          int n_chunks_max,
                                                          unsigned* __restrict__ counters,
                                                          float* __restrict__ part,
                                                          u16* __restrict__ out) {
  __shared__ float sm_m[4][16], sm_l[4][16];
  __shared__ float sm_o[4][16][HEAD_DIM + 4];
  __shared__ float sm_f[MAX_DECODE_CHUNKS][16];
  __shared__ float sm_L[16];
  __shared__ int sm_last;
  const int chunk = blockIdx.x, g = blockIdx.y, bseq = blockIdx.z;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int n_rep = H / KV;
  const int ctx = b.ctx_lens[bseq];
  const int n_pages = (ctx + KV_PAGE - 1) / KV_PAGE;
  const int cp = 4 * ppw;
  const int nc = (n_pages + cp - 1) / cp;
  if (chunk >= nc) return;  // uniform over the workgroup
  const int tok = b.seq_start[bseq + 1] - 1;
  const int hn = lane & 15;
  bf16x8 qf[4];
  if (hn < n_rep) {
    const u16* qp = q + ((int64_t)tok * H + g * n_rep + hn) * HEAD_DIM + 8 * (lane >> 4);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) qf[ks] = *(const bf16x8*)(qp + ks * 32);
  } else {
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) qf[ks] = as_bf16x8(u16x8{0, 0, 0, 0, 0, 0, 0, 0});
  }
  float m_i = -INFINITY, l_i = 0.f;
  f32x4 o[8];
#pragma unroll
  for (int db = 0; db < 8; ++db) o[db] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int* bt = b.block_table + (int64_t)bseq * b.max_pages;
  const int p0 = chunk * cp + wave * ppw;
  const int p1 = min(n_pages, p0 + ppw);
  for (int pi = p0; pi < p1; ++pi) {
    const int phys = bt[pi];
    const u16* kblk = kv + ((int64_t)(phys * 2 + 0) * KV + g) * KV_BLOCK_ELEMS;
    const u16* vblk = kv + ((int64_t)(phys * 2 + 1) * KV + g) * KV_BLOCK_ELEMS;
    attend_page(kblk, vblk, qf, pi * KV_PAGE, ctx - 1, scale_log2, m_i, l_i, o, lane);
  }
  // merge the 4 waves of this chunk through LDS
  if (lane < 16) {
    sm_m[wave][lane] = m_i;
    sm_l[wave][lane] = l_i;
  }
#pragma unroll
  for (int db = 0; db < 8; ++db)
#pragma unroll
    for (int r = 0; r < 4; ++r) sm_o[wave][hn][db * 16 + 4 * (lane >> 4) + r] = o[db][r];
  __syncthreads();
  u16* op = out + (int64_t)tok * H * HEAD_DIM + (int64_t)g * n_rep * HEAD_DIM;
  const int stride = n_rep * PART_STRIDE;
  float* base = part + ((int64_t)bseq * KV + g) * n_chunks_max * stride;
  for (int idx = threadIdx.x; idx < n_rep * HEAD_DIM; idx += 256) {
    const int n = idx / HEAD_DIM, d = idx % HEAD_DIM;
    const float M = fmaxf(fmaxf(sm_m[0][n], sm_m[1][n]), fmaxf(sm_m[2][n], sm_m[3][n]));
    float acc = 0.f, L = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const float f = exp2f(sm_m[w][n] - M);
      acc += sm_o[w][n][d] * f;
      L += sm_l[w][n] * f;
    }
    if (nc == 1) {
      op[n * HEAD_DIM + d] = f2bf(acc / L);
    } else {
      // write-through (sc1) partial stores: visible chip-wide once drained, no release fence
      float* pc = base + (int64_t)chunk * stride + n * PART_STRIDE;
      __hip_atomic_store(pc + d, acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (d == 0) {
        __hip_atomic_store(pc + HEAD_DIM, M, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(pc + HEAD_DIM + 1, L, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  if (nc == 1) return;
  // publish the partial (every storing wave drains, then one ticket); the last chunk merges
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev =
        __hip_atomic_fetch_add(&counters[bseq * KV + g], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    sm_last = (prev == (unsigned)(nc - 1));
    if (sm_last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(&counters[bseq * KV + g], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  if (!sm_last) return;
  // per-chunk scale factors f[c][n] = 2^(m_c - M_n) and the normaliser L_n
  for (int idx = threadIdx.x; idx < nc * n_rep; idx += 256) {
    const int c = idx / n_rep, n = idx % n_rep;
    sm_f[c][n] = base[(int64_t)c * stride + n * PART_STRIDE + HEAD_DIM];
  }
  __syncthreads();
  if (threadIdx.x < n_rep) {
    const int n = threadIdx.x;
    float M = -INFINITY;
    for (int c = 0; c < nc; ++c) M = fmaxf(M, sm_f[c][n]);
    float L = 0.f;
    for (int c = 0; c < nc; ++c) {
      const float f = exp2f(sm_f[c][n] - M);
      sm_f[c][n] = f;
      L += base[(int64_t)c * stride + n * PART_STRIDE + HEAD_DIM + 1] * f;
    }
    sm_L[n] = L;
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < n_rep * HEAD_DIM; idx += 256) {
    const int n = idx / HEAD_DIM, d = idx % HEAD_DIM;
    const float* pc = base + n * PART_STRIDE + d;
    float acc = 0.f;
#pragma unroll 8
    for (int c = 0; c < nc; ++c) acc += pc[(int64_t)c * stride] * sm_f[c][n];
    op[n * HEAD_DIM + d] = f2bf(acc / sm_L[n]);
  }
}

static int decode_ppw(int B, int KV, int max_ctx) {
  static int env = -2;
  if (env == -2) {
    const char* e = getenv("INFERD_DECODE_PPW");
    env = e ? atoi(e) : -1;
  }
  const int n_pages = (max_ctx + KV_PAGE - 1) / KV_PAGE;
  // ~2 four-wave workgroups per CU (512) over the (seq, kv-head, page) stream: measured on
  // B=16 x 2.1k ctx x 8 kv heads, 1 page/wave 31.8 us, 2: 29.9, 4: 28.2, 8: 33.7
  int ppw = env > 0 ? env : (B * KV * n_pages + 4 * 512 - 1) / (4 * 512);
  if (ppw < 1) ppw = 1;
  // chunks of 4*ppw pages; at most MAX_DECODE_CHUNKS chunks per sequence
  const int min_ppw = (n_pages + 4 * MAX_DECODE_CHUNKS - 1) / (4 * MAX_DECODE_CHUNKS);
  return ppw < min_ppw ? min_ppw : ppw;
}

size_t attn_decode_ws_bytes(int B, int H, int max_ctx) {
  // worst case over kv-head counts (KV <= H): MAX_DECODE_CHUNKS chunks of n_rep heads
  return DECODE_COUNTER_BYTES + (size_t)B * H * MAX_DECODE_CHUNKS * PART_STRIDE * sizeof(float);
}

void launch_attn_decode(const u16* q, const u16* kv_layer, const AttnBatch& b, int H, int KV,
                        float scale, u16* out, float* ws, hipStream_t s) {
  const int ppw = decode_ppw(b.B, KV, b.max_ctx);
  const int n_pages = (b.max_ctx + KV_PAGE - 1) / KV_PAGE;
  const int n_chunks = (n_pages + 4 * ppw - 1) / (4 * ppw);
  unsigned* counters = (unsigned*)ws;
  float* part = (float*)((char*)ws + DECODE_COUNTER_BYTES);
  hipLaunchKernelGGL(attn_decode_kernel, dim3(n_chunks, KV, b.B), dim3(256), 0, s, q, kv_layer, b, H, KV, ppw,
                     scale * LOG2E, n_chunks, counters, part, out);
}

// ------------------------------------------------------------------ prefill (causal)
// grid (ceil(max_q_len/128), H, B), 4 waves.  The workgroup owns 128 query rows of one head;
// wave w owns rows [32w, 32w+32) as two 16-row MFMA column blocks.  Every K/V page (K 16 KiB
// + V 16 KiB of this kv head) is staged ONCE per workgroup into double-buffered LDS with
// global_load_lds_dwordx4 (32 x 1 KiB pieces, 8 per wave) while the previous page is being
// consumed; the page layout is already fragment-ordered, so every fragment read is
// lds[tile * 1 KiB + lane * 16] (contiguous, bank-conflict free), and each K/V fragment feeds
// the MFMAs of both column blocks.  Waves whose rows all precede a page skip its compute but
// keep the barriers.
__device__ __forceinline__ void prefill_page_lds(const char* __restrict__ lds, const bf16x8 (&qf)[2][4],
                                                 int page_tok0, const int (&lim)[2], float scale_log2,
                                                 float (&m_i)[2], float (&l_i)[2], f32x4 (&o)[2][8], int lane) {
  f32x4 sc[2][4];
#pragma unroll
  for (int nb = 0; nb < 2; ++nb)
#pragma unroll
    for (int tb = 0; tb < 4; ++tb) sc[nb][tb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int tb = 0; tb < 4; ++tb)
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const bf16x8 kf = *(const bf16x8*)(lds + (tb * 4 + ks) * 1024 + lane * 16);
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) sc[nb][tb] = mfma16(kf, qf[nb][ks], sc[nb][tb]);
    }
  bf16x8 pf[2][2];
#pragma unroll
  for (int nb = 0; nb < 2; ++nb) {
    float pmax = -INFINITY;
#pragma unroll
    for (int tb = 0; tb < 4; ++tb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int t = page_tok0 + tb * 16 + 4 * (lane >> 4) + r;
        const float s = (t <= lim[nb]) ? sc[nb][tb][r] * scale_log2 : -INFINITY;
        sc[nb][tb][r] = s;
        pmax = fmaxf(pmax, s);
      }
    pmax = fmaxf(pmax, __shfl_xor(pmax, 16));
    pmax = fmaxf(pmax, __shfl_xor(pmax, 32));
    const float m_new = fmaxf(m_i[nb], pmax);
    const float alpha = exp2f(m_i[nb] - m_new);
    float psum = 0.f;
#pragma unroll
    for (int tb = 0; tb < 4; ++tb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = exp2f(sc[nb][tb][r] - m_new);
        sc[nb][tb][r] = p;
        psum += p;
      }
    psum += __shfl_xor(psum, 16);
    psum += __shfl_xor(psum, 32);
    l_i[nb] = l_i[nb] * alpha + psum;
    m_i[nb] = m_new;
#pragma unroll
    for (int db = 0; db < 8; ++db) o[nb][db] *= alpha;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pf[nb][kt][j] = (__bf16)sc[nb][2 * kt][j];
        pf[nb][kt][4 + j] = (__bf16)sc[nb][2 * kt + 1][j];
      }
  }
#pragma unroll
  for (int kt = 0; kt < 2; ++kt)
#pragma unroll
    for (int db = 0; db < 8; ++db) {
      const bf16x8 vf = *(const bf16x8*)(lds + 16384 + (kt * 8 + db) * 1024 + lane * 16);
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) o[nb][db] = mfma16(vf, pf[nb][kt], o[nb][db]);
    }
}

__global__ __launch_bounds__(256, 2) void attn_prefill_kernel(const u16* __restrict__ q,
                                                           const u16* __restrict__ kv,
                                                           AttnBatch b, int H, int KV,
                                                           float scale_log2,
                                                           u16* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) char lds[2 * 32768];
  const int bseq = blockIdx.z, h = blockIdx.y;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int n_rep = H / KV, g = h / n_rep;
  const int t0 = b.seq_start[bseq];
  const int T = b.seq_start[bseq + 1] - t0;
  const int qb0 = blockIdx.x * 128;
  if (qb0 >= T) return;  // uniform over the workgroup
  bf16x8 qf[2][4];
  int lim[2], tokrow[2];
  bool valid[2];
#pragma unroll
  for (int nb = 0; nb < 2; ++nb) {
    const int row = qb0 + wave * 32 + nb * 16 + (lane & 15);
    valid[nb] = row < T;
    tokrow[nb] = t0 + (valid[nb] ? row : T - 1);
    lim[nb] = b.positions[tokrow[nb]];
    const u16* qp = q + ((int64_t)tokrow[nb] * H + h) * HEAD_DIM + 8 * (lane >> 4);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) qf[nb][ks] = *(const bf16x8*)(qp + ks * 32);
  }
  // pages: up to the workgroup's last row; a wave computes up to its own last row
  const int wg_last = b.positions[t0 + min(qb0 + 127, T - 1)];
  const int wave_first_row = qb0 + wave * 32;
  const int wave_last = wave_first_row < T ? b.positions[t0 + min(wave_first_row + 31, T - 1)] : -1;
  const int n_pages = wg_last / KV_PAGE + 1;
  const int* bt = b.block_table + (int64_t)bseq * b.max_pages;
  auto stage = [&](int buf, int pi) {
    const int phys = bt[pi];
    const u16* kblk = kv + ((int64_t)(phys * 2 + 0) * KV + g) * KV_BLOCK_ELEMS;
    const u16* vblk = kv + ((int64_t)(phys * 2 + 1) * KV + g) * KV_BLOCK_ELEMS;
    char* base = lds + buf * 32768;
#pragma unroll
    for (int pc = 0; pc < 8; ++pc) {
      const int piece = wave * 8 + pc;  // 0..15 K tiles, 16..31 V tiles
      const u16* src = (piece < 16 ? kblk + piece * 512 : vblk + (piece - 16) * 512) + lane * 8;
      __builtin_amdgcn_global_load_lds((const void*)src, (void*)(base + piece * 1024), 16, 0, 0);
    }
  };
  float m_i[2] = {-INFINITY, -INFINITY}, l_i[2] = {0.f, 0.f};
  f32x4 o[2][8];
#pragma unroll
  for (int nb = 0; nb < 2; ++nb)
#pragma unroll
    for (int db = 0; db < 8; ++db) o[nb][db] = f32x4{0.f, 0.f, 0.f, 0.f};
  stage(0, 0);
  __syncthreads();
  for (int pi = 0; pi < n_pages; ++pi) {
    const int cur = pi & 1;
    if (pi + 1 < n_pages) stage(cur ^ 1, pi + 1);
    if (pi * KV_PAGE <= wave_last)
      prefill_page_lds(lds + cur * 32768, qf, pi * KV_PAGE, lim, scale_log2, m_i, l_i, o, lane);
    __syncthreads();  // next page landed (vmcnt(0)) and everyone is done with this buffer
  }
#pragma unroll
  for (int nb = 0; nb < 2; ++nb) {
    if (!valid[nb]) continue;
    const float inv = 1.0f / l_i[nb];
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

void launch_attn_prefill(const u16* q, const u16* kv_layer, const AttnBatch& b, int H, int KV,
                         float scale, u16* out, hipStream_t s) {
  dim3 g((b.max_q_len + 127) / 128, H, b.B);
  hipLaunchKernelGGL(attn_prefill_kernel, g, dim3(256), 0, s, q, kv_layer, b, H, KV,
                     scale * LOG2E, out);
}
