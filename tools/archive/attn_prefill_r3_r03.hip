// Archived in round 4 from inferd_amd/csrc/attention.hip (INFERD_ATTN_PREFILL=6): bit-identical
// to the default prefill attention and slower than the 48-row kernel.  Not built;
// it needs attention.hip's prefill_page_s / prefill_page_pv helpers of the round-3 tree (git 84f0988).
// Three workgroups per CU (3 waves per SIMD): the same 4-wave workgroup with 32 rows per wave
// (157 VGPRs under these launch bounds) and a 48 KiB LDS ring of three 16 KiB half-page slots
// (K or V of one page; half-page u = 2 page + {0: K, 1: V} lives in slot u % 3).  Per page two
// barriers: after S + softmax (K(i) consumed: its slot takes V(i+1)) and after P.V (V(i)
// consumed: its slot takes K(i+2)); each barrier first waits for this wave's pieces of the half
// the next phase reads (vmcnt leaves the one half issued after it in flight).
template <int NB>
__global__ __launch_bounds__(256, 3) void attn_prefill_r3_kernel(const u16* __restrict__ q,
                                                              const u16* __restrict__ kv, AttnBatch b, int H,
                                                              int KV, float scale_log2, u16* __restrict__ out,
                                                              int order) {
  constexpr int QB = 64 * NB, RW = 16 * NB;
  __shared__ __attribute__((aligned(16))) char lds[3 * 16384];
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
  if (qb >= nqb) return;
  const int qb0 = qb * QB;
  bf16x8 qf[NB][4];
  int lim[NB], tokrow[NB];
  bool valid[NB];
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
  const int wg_last = b.positions[t0 + min(qb0 + QB - 1, T - 1)];
  const int wave_first_row = qb0 + wave * RW;
  const int wave_last = wave_first_row < T ? b.positions[t0 + min(wave_first_row + RW - 1, T - 1)] : -1;
  int wave_min_lim = lim[0];
#pragma unroll
  for (int nb = 1; nb < NB; ++nb) wave_min_lim = min(wave_min_lim, lim[nb]);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) wave_min_lim = min(wave_min_lim, __shfl_xor(wave_min_lim, off));
  const int n_pages = wg_last / KV_PAGE + 1;
  const int n_half = 2 * n_pages;
  typedef const __attribute__((address_space(4))) int* cptr;
  typedef __attribute__((address_space(3))) void* lds_ptr;
  const cptr bt = (cptr)(b.block_table + (int64_t)bseq * b.max_pages);
  const int swave = __builtin_amdgcn_readfirstlane(wave);
  // half-page u -> slot u % 3: this wave's 4 of its 16 pieces
  auto stage = [&](int u) {
    const int pi = u >> 1, kind = u & 1;
    const __amdgpu_buffer_rsrc_t pg_rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void*)(kv + kv_block(bt[pi], 0, g, KV)), 0, 2 * KV_BLOCK_ELEMS * 2, 0x00020000);
    char* base = lds + (u % 3) * 16384;
#pragma unroll
    for (int pc = 0; pc < 4; ++pc) {
      const int piece = swave * 4 + pc;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(pg_rsrc, (lds_ptr)(base + piece * 1024), 16, lane * 16,
                                               (kind * 16 + piece) * 1024, 0, 0);
    }
  };
  float m_i[NB], l_i[NB];
  f32x4 o[NB][8];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    m_i[nb] = -INFINITY;
    l_i[nb] = 0.f;
#pragma unroll
    for (int db = 0; db < 8; ++db) o[nb][db] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  // prologue: K0, V0, K1 in flight; K0 must land before S(0): vmcnt leaves V0 and K1
  stage(0);
  stage(1);
  if (n_half > 2) {
    stage(2);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  }
  raw_barrier();  // (__syncthreads() would drain the half-pages left in flight)
  bf16x8 pf[NB][2];
  for (int pi = 0; pi < n_pages; ++pi) {
    const int tok0 = pi * KV_PAGE;
    const char* kl = lds + ((2 * pi) % 3) * 16384;
    const char* vl = lds + ((2 * pi + 1) % 3) * 16384;
    const bool live = tok0 <= wave_last;
    if (tok0 + KV_PAGE - 1 <= wave_min_lim)
      prefill_page_s<false, NB>(kl, qf, tok0, lim, scale_log2, m_i, l_i, o, lane, pf);
    else if (live)
      prefill_page_s<true, NB>(kl, qf, tok0, lim, scale_log2, m_i, l_i, o, lane, pf);
    // B1: V(i) landed (in flight after it: K(i+1) if issued); K(i)'s slot takes V(i+1)
    if (2 * pi + 2 < n_half)
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    raw_barrier();
    if (2 * pi + 3 < n_half) stage(2 * pi + 3);
    if (live) prefill_page_pv<NB>(vl, pf, o, lane);
    // B2: K(i+1) landed (in flight after it: V(i+1) if issued); V(i)'s slot takes K(i+2)
    if (2 * pi + 3 < n_half)
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    raw_barrier();
    if (2 * pi + 4 < n_half) stage(2 * pi + 4);
  }
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    const float inv = 1.0f / sum_q4(l_i[nb]);
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

