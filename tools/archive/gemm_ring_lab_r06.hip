// ARCHIVED LAB (round 6): gemm_w4_kernel's K-loop on a ring of W4_RING LDS
// buffers of 32-deep K-steps, spliced into gemm_w4_kernel in place of its two 64-deep buffers
// (lds[W4_RING * 32768]) and built with tools/build_probes.sh gemm.hip ring5='-DW4_RING=5'.
// Result (profiles/r06/gemm_ring_ab.txt, span_ab_ring5.txt): bit-identical; down 1557.5 us
// (product) vs 1762.6 (4 buffers, 2 steps of cover) vs 1877.2 (5 buffers, 3 steps of cover); o
// 526.0 vs 606.2 vs 665.8; in a 2-layer config-5 stage down 1620 vs 2041 us.  The deeper ring is
// the slower one: down's K-loop is not bound by the latency cover of its LDS refills.
#ifdef W4_RING
  // ---- LAB (tools/build_probes.sh gemm.hip ring5='-DW4_RING=5'): the same
  // tile and accumulators on a ring of W4_RING LDS buffers of 32-deep K-steps (32 KiB each: A image
  // [256 rows][64 B] with a 16-B chunk XOR swizzle, B image [16 n-tiles][1 KiB]), W4_RING - 2
  // steps of HBM latency cover instead of one 64-deep step.  Step s lives in buffer s % NB; its
  // fragments are read during iteration s - 1 and consumed by iteration s's 64 MFMAs (in K order,
  // so the accumulation order -- and every output bit -- is gemm_w4_kernel's).
  f32x4 acc[8][8];
  {
    constexpr int NB = W4_RING;
    const int nK = KT / nsl;  // 32-deep K-steps of this slice
    const int k0 = slice * nK;
    const int wv = __builtin_amdgcn_readfirstlane(wave);
    const char* a_base = (const char*)(A + (int64_t)m0 * lda + k0 * 32);
    unsigned a_voff[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {  // wave rows 64 wave + 16 p + lane / 4, image chunk lane % 4
      const int i = 64 * wave + 16 * p + (lane >> 2);
      const int rr = (m0 + i < M ? i : M - 1 - m0);
      const int chunk = (lane & 3) ^ ((i >> 2) & 3);
      a_voff[p] = (unsigned)(rr * lda * 2 + chunk * 16);
    }
    int64_t b_soff[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int j = 4 * wv + p;  // image n-tile
      int gnt;
      if constexpr (EPI == EPI_SILU) {
        const int w = j >> 3, jj = j & 7;
        gnt = (jj < 4 ? 0 : n_tiles_w / 2) + n0 / 16 + 4 * w + (jj & 3);
      } else {
        gnt = n0 / 16 + j;
      }
      b_soff[p] = ((int64_t)gnt * KT + k0) * 1024;
    }
    const __amdgpu_buffer_rsrc_t a_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)a_base, 0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t b_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)Wp, 0, 0x7fffffff, 0x00020000);
    typedef __attribute__((address_space(3))) void* lds_ptr;
    auto issue = [&](int p, int t) {  // piece p (0-3 A, 4-7 B) of K-step t into buffer t % NB
      char* base = lds + (t % NB) * 32768;
      if (p < 4)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(a_rsrc, (lds_ptr)(base + (4 * wv + p) * 1024), 16, a_voff[p], t * 64, 0,
                                                 0);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(b_rsrc, (lds_ptr)(base + 16384 + (4 * wv + p - 4) * 1024), 16,
                                                 lane * 16, (int)(b_soff[p - 4] + (int64_t)t * 1024), 0, 0);
    };
    const int arow = wr * 128 + (lane & 15);
    const int a_off = arow * 64 + 16 * ((lane >> 4) ^ ((arow >> 2) & 3));
    const int b_off = 16384 + (8 * wc) * 1024 + lane * 16;
    bf16x8 fa[2][8], fb[2][8];
    auto read_f = [&](int f, int g, int t) {  // fragment g (0-7 A, 8-15 B) of step t into set f
      const char* base = lds + (t % NB) * 32768;
      if (g < 8)
        fa[f][g] = *(const bf16x8*)(base + a_off + g * 1024);
      else
        fb[f][g - 8] = *(const bf16x8*)(base + b_off + (g - 8) * 1024);
    };
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto fence = [&]() {  // as acc_fence below: 16 wait states, every accumulator redefined after them
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
    fence();
    // prologue: steps 0 .. NB-2 in flight; steps 0 and 1 landed; step 0's fragments read
    for (int t = 0; t < NB - 1 && t < nK; ++t)
#pragma unroll
      for (int p = 0; p < 8; ++p) issue(p, t);
    if (nK >= NB - 1)
      vm_wait<8 * (NB - 3)>();
    else
      vm_wait<0>();
    raw_barrier();
#pragma unroll
    for (int g = 0; g < 16; ++g) read_f(0, g, 0);
    auto step = [&](auto F, int t, bool more, bool steady) {
      constexpr int f = decltype(F)::value;
      // 64 MFMAs on fragment set f (step t); the next step's fragments into set f ^ 1 during the
      // first 16, step t + NB - 1's pieces into buffer (t - 1) % NB (read by every wave before the
      // previous barrier) during the next 8 groups of 4
#pragma unroll
      for (int x = 0; x < 64; ++x) {
        if (x == 0) __builtin_amdgcn_s_waitcnt(0xC07F);  // set f's reads landed
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0"
                     : "+a"(acc[x >> 3][x & 7])
                     : "v"(fb[f][x & 7]), "v"(fa[f][x >> 3]));
        if (more && x < 16) read_f(f ^ 1, x, t + 1);
        if (steady && x >= 16 && x < 48 && (x & 3) == 0) issue((x - 16) >> 2, t + NB - 1);
        __builtin_amdgcn_sched_barrier(0);
      }
      // step t + 2 landed (the younger steps' pieces may still fly), visible to every wave
      if (steady)
        vm_wait<8 * (NB - 3)>();
      else
        vm_wait<0>();
      raw_barrier();
    };
    int t = 0;
    for (; t + 1 < nK; t += 2) {
      step(std::integral_constant<int, 0>{}, t, true, t + NB - 1 < nK);
      step(std::integral_constant<int, 1>{}, t + 1, t + 2 < nK, t + NB < nK);
    }
    if (t < nK) step(std::integral_constant<int, 0>{}, t, false, false);
    fence();
  }
