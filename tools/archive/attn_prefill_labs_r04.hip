// Archived in round 4 from inferd_amd/csrc/attention.hip: prefill attention lab kernels measured
// against the 4-wave kernel (tools/attn_ab.py, Qwen3-32B dims, T = 8192, one box,
// profiles/r04/attn_ab.txt; base = round-3 default 1019.6 us, with the softmax cuts 944.2 us):
//   attn_prefill8_kernel      8 waves, two per SIMD, staggered segments: 1089.5 us (1094.4 with
//                             the softmax cuts, 1088.4 with static priority for waves 4-7)
//   attn_prefill_pipe_kernel  4 waves, S(i+1) beside page i's softmax: 1044.8 us (1039.9 with the
//                             steady state as one interleaved block)
// Not built; they need attention.hip's PfState / prefill helpers of the round-4 tree.
// 8 waves, two per SIMD, one workgroup per CU (PF_KERNEL=8, lab).  The workgroup owns 256 query
// rows of one head; wave w (half hf = w >> 2, k = w & 3) owns rows 64 k + 32 hf .. +31 (two 16-row
// column blocks), so the two waves sharing a SIMD (w, w + 4) have neighbouring rows.  Per page i
// two segments separated by raw barriers:
//   seg1(i): S(i) = K(i) q' - m (16 MFMA chains, k-slice outermost) and O += V(i-1) P(i-1) (+ the
//            row-sum MFMAs): matrix work only;
//   seg2(i): softmax of page i (VALU), LDS-DMA of K(i+3) / V(i+2), counted wait.
// Waves 4-7 run one barrier behind waves 0-3, so on every SIMD one wave is in its matrix segment
// while its partner is in its softmax segment (MI355X_MICROARCH.md, two waves per SIMD).  With
// the softmax cuts (PF_CUTS) the softmax segment is shorter than the partner's matrix segment.
// K and V each have a 4-slot ring of 16 KiB half pages; slot reuse: K(i+3) goes to K(i-1)'s slot,
// V(i+2) to V(i-2)'s, both last read one segment earlier by the lagging half.
__global__ __launch_bounds__(512, 1) void attn_prefill8_kernel(const u16* __restrict__ q,
                                                             const u16* __restrict__ kv, AttnBatch b, int H,
                                                             int KV, float scale_log2, u16* __restrict__ out) {
  constexpr int NB = 2;
  __shared__ __attribute__((aligned(16))) char lds[8 * 16384];
  const int bseq = blockIdx.y;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int hf = wave >> 2, kw = wave & 3;
  const int n_rep = H / KV;
  const int mqb = (b.max_q_len + 255) / 256;
  int h, qbi;
  if (gridDim.x % 8 == 0) {
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
  const int nqb = (T + 255) / 256;
  const int qbk = mqb - 1 - qbi;  // heaviest blocks dispatch first
  if (qbk >= nqb) return;         // uniform over the workgroup
  const int qb0 = qbk * 256;
  const int row0 = qb0 + kw * 64 + hf * 32;
  bf16x8 qf[NB][4];
  int lim[NB], tokrow[NB];
  bool valid[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    const int row = row0 + nb * 16 + (lane & 15);
    valid[nb] = row < T;
    tokrow[nb] = t0 + (valid[nb] ? row : T - 1);
    lim[nb] = b.positions[tokrow[nb]];
    const u16* qp = q + ((int64_t)tokrow[nb] * H + h) * HEAD_DIM + 8 * (lane >> 4);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) qf[nb][ks] = *(const bf16x8*)(qp + ks * 32);
  }
  if constexpr (PF_CUTS) {
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
#pragma unroll
        for (int j = 0; j < 8; ++j) qf[nb][ks][j] = (__bf16)((float)qf[nb][ks][j] * scale_log2);
  }
  const int wave_last = row0 < T ? b.positions[t0 + min(row0 + 31, T - 1)] : -1;
  int wave_min_lim = min(lim[0], lim[1]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) wave_min_lim = min(wave_min_lim, __shfl_xor(wave_min_lim, o));
  const int n_pages = b.positions[t0 + min(qb0 + 255, T - 1)] / KV_PAGE + 1;
  typedef const __attribute__((address_space(4))) int* cptr;
  typedef __attribute__((address_space(3))) void* lds_ptr;
  const cptr bt = (cptr)(b.block_table + (int64_t)bseq * b.max_pages);
  const int swave = __builtin_amdgcn_readfirstlane(wave);
  // this wave's 2 of the 16 1-KiB pieces of K (kind 0) or V (kind 1) of page j (clamped to a
  // real page past the end: every segment issues the same count, so the waits stay counted;
  // the clamped copy lands in a free slot and is never read)
  auto issue = [&](int kind, int j) {
    const int jj = j < n_pages ? j : n_pages - 1;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(kv + kv_block(bt[jj], 0, g, KV)), 0, 2 * KV_BLOCK_ELEMS * 2, 0x00020000);
    char* dst = lds + (kind * 4 + (j & 3)) * 16384;
#pragma unroll
    for (int pc = 0; pc < 2; ++pc) {
      const int piece = swave * 2 + pc;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr)(dst + piece * 1024), 16, lane * 16,
                                               (kind * 16 + piece) * 1024, 0, 0);
    }
  };
  float m_i[NB], l_i[NB];
  PfState ps_[NB];
  f32x4 o[NB][8], sc[NB][4];
  bf16x8 pf[NB][2];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    m_i[nb] = -INFINITY;
    l_i[nb] = 0.f;
    ps_[nb].negm = f32x4{0.f, 0.f, 0.f, 0.f};
    ps_[nb].l = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int db = 0; db < 8; ++db) o[nb][db] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  issue(0, 0);
  issue(0, 1);
  issue(1, 0);
  issue(0, 2);
  issue(1, 1);
  vm_wait<0>();
  raw_barrier();
  if (hf) raw_barrier();  // stagger: waves 4-7 one segment behind
#ifdef PF_PRIO
  // static priority for the second-dispatched half (MI355X_MICROARCH.md two waves per SIMD, item 4)
  if (__builtin_amdgcn_readfirstlane(threadIdx.x) >= 256) __builtin_amdgcn_s_setprio(1);
#endif
  for (int i = 0; i <= n_pages; ++i) {
    const bool do_s = i < n_pages && i * KV_PAGE <= wave_last;
    const bool do_pv = i > 0 && (i - 1) * KV_PAGE <= wave_last;
    // ---------------- seg1(i): S(i) and P.V(i-1), matrix work only
    if (do_s) {
      const char* kb = lds + (i & 3) * 16384 + lane * 16;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
#pragma unroll
        for (int tb = 0; tb < 4; ++tb) {
          const bf16x8 kf = *(const bf16x8*)(kb + (tb * 4 + ks) * 1024);
#pragma unroll
          for (int nb = 0; nb < NB; ++nb) {
            f32x4 c0 = f32x4{0.f, 0.f, 0.f, 0.f};
            if (PF_CUTS && i > 0) c0 = ps_[nb].negm;
            sc[nb][tb] = mfma16(kf, qf[nb][ks], ks ? sc[nb][tb] : c0);
          }
        }
    }
    if (do_pv) {
      const char* vb = lds + (4 + ((i - 1) & 3)) * 16384 + lane * 16;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
        for (int db = 0; db < 8; ++db) {
          const bf16x8 vf = *(const bf16x8*)(vb + (kt * 8 + db) * 1024);
#pragma unroll
          for (int nb = 0; nb < NB; ++nb) o[nb][db] = mfma16(vf, pf[nb][kt], o[nb][db]);
        }
        if constexpr (PF_CUTS) {
          bf16x8 ones;
#pragma unroll
          for (int j = 0; j < 8; ++j) ones[j] = (__bf16)1.0f;
#pragma unroll
          for (int nb = 0; nb < NB; ++nb) ps_[nb].l = mfma16(ones, pf[nb][kt], ps_[nb].l);
        }
      }
    }
    if (i == n_pages) break;
    raw_barrier();
    // ---------------- seg2(i): staging, softmax(i), counted wait
    issue(0, i + 3);
    issue(1, i + 2);
    if (do_s) {
      const int tok0 = i * KV_PAGE;
      const bool mask = tok0 + KV_PAGE - 1 > wave_min_lim;
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        if (mask) {
#pragma unroll
          for (int tb = 0; tb < 4; ++tb)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int t = tok0 + tb * 16 + 4 * (lane >> 4) + r;
              sc[nb][tb][r] = (t <= lim[nb]) ? sc[nb][tb][r] : -INFINITY;
            }
        }
        float pm[4];
#pragma unroll
        for (int tb = 0; tb < 4; ++tb)
          pm[tb] = fmaxf(fmaxf(sc[nb][tb][0], sc[nb][tb][1]), fmaxf(sc[nb][tb][2], sc[nb][tb][3]));
        const float pmax = max_q4(fmaxf(fmaxf(pm[0], pm[1]), fmaxf(pm[2], pm[3])));
        if constexpr (PF_CUTS) {
          float shift = 0.f;
          if (i == 0) {
            shift = pmax;
            m_i[nb] = pmax;
            ps_[nb].negm = f32x4{-pmax, -pmax, -pmax, -pmax};
          } else if (__builtin_amdgcn_ballot_w64(pmax > RESCALE_THR)) {
            shift = fmaxf(pmax, 0.f);
            const float alpha = exp2_raw(-shift);
            ps_[nb].l *= alpha;
#pragma unroll
            for (int db = 0; db < 8; ++db) o[nb][db] *= alpha;
            m_i[nb] += shift;
            ps_[nb].negm = f32x4{-m_i[nb], -m_i[nb], -m_i[nb], -m_i[nb]};
          }
          if (shift != 0.f) {
#pragma unroll
            for (int tb = 0; tb < 4; ++tb) sc[nb][tb] -= shift;
          }
#pragma unroll
          for (int tb = 0; tb < 4; ++tb)
#pragma unroll
            for (int r = 0; r < 4; ++r) sc[nb][tb][r] = exp2_raw(sc[nb][tb][r]);
        } else {
          const float m_new = fmaxf(m_i[nb], pmax * scale_log2);
          if (__builtin_amdgcn_ballot_w64(m_new > m_i[nb] + RESCALE_THR)) {
            const float alpha = exp2_raw(m_i[nb] - m_new);
            l_i[nb] *= alpha;
#pragma unroll
            for (int db = 0; db < 8; ++db) o[nb][db] *= alpha;
            m_i[nb] = m_new;
          }
          const float mneg = -m_i[nb];
          float ps[4];
#pragma unroll
          for (int tb = 0; tb < 4; ++tb) {
#pragma unroll
            for (int r = 0; r < 4; ++r) sc[nb][tb][r] = exp2_raw(fmaf(sc[nb][tb][r], scale_log2, mneg));
            ps[tb] = (sc[nb][tb][0] + sc[nb][tb][1]) + (sc[nb][tb][2] + sc[nb][tb][3]);
          }
          l_i[nb] += (ps[0] + ps[1]) + (ps[2] + ps[3]);
        }
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            pf[nb][kt][j] = (__bf16)sc[nb][2 * kt][j];
            pf[nb][kt][4 + j] = (__bf16)sc[nb][2 * kt + 1][j];
          }
      }
    }
    // K(i+1) and V(i) (read in seg1(i+1)) landed: the leading half leaves its two newer
    // groups in flight, the lagging half (one segment later at every barrier) one
    if (hf)
      vm_wait<4>();
    else
      vm_wait<8>();
    raw_barrier();
  }
  if (!hf) raw_barrier();  // close the stagger
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    const float inv = 1.0f / (PF_CUTS ? ps_[nb].l[0] : sum_q4(l_i[nb]));
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

// Software-pipelined 4-wave body (PF_KERNEL=5, lab): 2 workgroups per CU, 32 query rows per wave
// (NB = 2), PF_CUTS softmax.  Iteration i of a wave: phase A issues S(i+1)'s MFMAs beside the
// exp2 / bf16 packing of page i; phase B issues P.V(i)'s MFMAs beside the mask / row max of page
// i+1, whose rescale (rare) is applied after them.  LDS: K and V rings of two 16 KiB half-page
// slots each; K(i+2) and V(i+1) are staged at the top of iteration i into the slots K(i) and
// V(i-1) left (both last read before the previous barrier) and waited at its bottom.
__global__ __launch_bounds__(256, 2) void attn_prefill_pipe_kernel(const u16* __restrict__ q,
                                                                 const u16* __restrict__ kv, AttnBatch b, int H,
                                                                 int KV, float scale_log2, u16* __restrict__ out) {
  constexpr int NB = 2, QB = 128, RW = 32;
  __shared__ __attribute__((aligned(16))) char lds[4 * 16384];  // K slots 0, 1; V slots 2, 3
  const int bseq = blockIdx.y;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int n_rep = H / KV;
  const int mqb = (b.max_q_len + QB - 1) / QB;
  int h, qbi;
  if (gridDim.x % 8 == 0) {
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
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int j = 0; j < 8; ++j) qf[nb][ks][j] = (__bf16)((float)qf[nb][ks][j] * scale_log2);
  }
  const int wg_last = b.positions[t0 + min(qb0 + QB - 1, T - 1)];
  const int wave_first_row = qb0 + wave * RW;
  const int wave_last = wave_first_row < T ? b.positions[t0 + min(wave_first_row + RW - 1, T - 1)] : -1;
  int wave_min_lim = min(lim[0], lim[1]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) wave_min_lim = min(wave_min_lim, __shfl_xor(wave_min_lim, o));
  const int n_pages = wg_last / KV_PAGE + 1;
  typedef const __attribute__((address_space(4))) int* cptr;
  typedef __attribute__((address_space(3))) void* lds_ptr;
  const cptr bt = (cptr)(b.block_table + (int64_t)bseq * b.max_pages);
  const int swave = __builtin_amdgcn_readfirstlane(wave);
  // this wave's 4 of the 16 pieces of K (kind 0) or V (kind 1) of page j into its slot
  auto stage = [&](int kind, int j) {
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(kv + kv_block(bt[j], 0, g, KV)), 0, 2 * KV_BLOCK_ELEMS * 2, 0x00020000);
    char* dst = lds + (kind * 2 + (j & 1)) * 16384;
#pragma unroll
    for (int pc = 0; pc < 4; ++pc) {
      const int piece = swave * 4 + pc;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr)(dst + piece * 1024), 16, lane * 16,
                                               (kind * 16 + piece) * 1024, 0, 0);
    }
  };
  float m_i[NB];
  PfState ps_[NB];
  f32x4 o[NB][8];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    m_i[nb] = 0.f;
    ps_[nb].negm = f32x4{0.f, 0.f, 0.f, 0.f};
    ps_[nb].l = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int db = 0; db < 8; ++db) o[nb][db] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  bf16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (__bf16)1.0f;
  // S(j) from K slot j & 1, C operand = -m (zero for page 0)
  auto s_mfma = [&](int j, f32x4 (&sc)[NB][4]) {
    const char* kb = lds + (j & 1) * 16384 + lane * 16;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int tb = 0; tb < 4; ++tb) {
        const bf16x8 kf = *(const bf16x8*)(kb + (tb * 4 + ks) * 1024);
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) sc[nb][tb] = mfma16(kf, qf[nb][ks], ks ? sc[nb][tb] : ps_[nb].negm);
      }
  };
  // mask + row max of page j's scores; rescale decision (o / l / m / negm updated) and the
  // scores shifted onto the new reference.  first: page 0 sets m.
  auto s_max = [&](int j, f32x4 (&sc)[NB][4], bool first) {
    const int tok0 = j * KV_PAGE;
    const bool mask = tok0 + KV_PAGE - 1 > wave_min_lim;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      if (mask) {
#pragma unroll
        for (int tb = 0; tb < 4; ++tb)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int t = tok0 + tb * 16 + 4 * (lane >> 4) + r;
            sc[nb][tb][r] = (t <= lim[nb]) ? sc[nb][tb][r] : -INFINITY;
          }
      }
      float pm[4];
#pragma unroll
      for (int tb = 0; tb < 4; ++tb)
        pm[tb] = fmaxf(fmaxf(sc[nb][tb][0], sc[nb][tb][1]), fmaxf(sc[nb][tb][2], sc[nb][tb][3]));
      const float pmax = max_q4(fmaxf(fmaxf(pm[0], pm[1]), fmaxf(pm[2], pm[3])));
      float shift = 0.f;
      if (first) {
        shift = pmax;
        m_i[nb] = pmax;
        ps_[nb].negm = f32x4{-pmax, -pmax, -pmax, -pmax};
      } else if (__builtin_amdgcn_ballot_w64(pmax > RESCALE_THR)) {
        shift = fmaxf(pmax, 0.f);
        const float alpha = exp2_raw(-shift);
        ps_[nb].l *= alpha;
#pragma unroll
        for (int db = 0; db < 8; ++db) o[nb][db] *= alpha;
        m_i[nb] += shift;
        ps_[nb].negm = f32x4{-m_i[nb], -m_i[nb], -m_i[nb], -m_i[nb]};
      }
      if (shift != 0.f) {
#pragma unroll
        for (int tb = 0; tb < 4; ++tb) sc[nb][tb] -= shift;
      }
    }
  };
  auto s_exp = [&](f32x4 (&sc)[NB][4], bf16x8 (&pf)[NB][2]) {
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          pf[nb][kt][j] = (__bf16)exp2_raw(sc[nb][2 * kt][j]);
          pf[nb][kt][4 + j] = (__bf16)exp2_raw(sc[nb][2 * kt + 1][j]);
        }
  };
  auto pv_mfma = [&](int j, const bf16x8 (&pf)[NB][2]) {
    const char* vb = lds + (2 + (j & 1)) * 16384 + lane * 16;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
      for (int db = 0; db < 8; ++db) {
        const bf16x8 vf = *(const bf16x8*)(vb + (kt * 8 + db) * 1024);
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) o[nb][db] = mfma16(vf, pf[nb][kt], o[nb][db]);
      }
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) ps_[nb].l = mfma16(ones, pf[nb][kt], ps_[nb].l);
    }
  };
  const bool live = wave_last >= 0;
  stage(0, 0);
  stage(1, 0);
  if (n_pages > 1) {
    stage(0, 1);
    stage(1, 1);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  raw_barrier();
  f32x4 sc[NB][4];
  if (live) {
    s_mfma(0, sc);
    s_max(0, sc, true);
  }
  for (int i = 0; i < n_pages; ++i) {
    // K(i) and V(i-1) slots are free (last read before the previous barrier)
    if (i + 2 < n_pages) stage(0, i + 2);
    if (i >= 1 && i + 1 < n_pages) stage(1, i + 1);
    const bool cur = live && i * KV_PAGE <= wave_last;
    const bool nxt = live && (i + 1) < n_pages && (i + 1) * KV_PAGE <= wave_last;
    bf16x8 pf[NB][2];
    f32x4 sn[NB][4];
#ifdef PF_PIPE_BLOCK
    if (cur && nxt) {
      // steady state: each phase one basic block, MFMAs interleaved with the other page's VALU
      __builtin_amdgcn_sched_barrier(0);
      s_mfma(i + 1, sn);
      s_exp(sc, pf);
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read (the 16 K fragments)
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
        __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);  // VALU (exp / pack)
      }
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
        __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);  // VALU
      }
      __builtin_amdgcn_sched_barrier(0);
      pv_mfma(i, pf);
      s_max(i + 1, sn, false);
    } else
#endif
    {
      // phase A: S(i+1) beside exp / packing of page i
      if (nxt) s_mfma(i + 1, sn);
      if (cur) s_exp(sc, pf);
      // phase B: P.V(i) beside the max of page i+1 (its rescale waits for P.V(i) by data dependence)
      if (cur) pv_mfma(i, pf);
      if (nxt) s_max(i + 1, sn, false);
    }
    if (nxt) {
#pragma unroll
      for (int nb = 0; nb < NB; ++nb)
#pragma unroll
        for (int tb = 0; tb < 4; ++tb) sc[nb][tb] = sn[nb][tb];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    raw_barrier();
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

