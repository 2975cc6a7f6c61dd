// ARCHIVE -- not built.  Superseded prefill GEMM bodies removed from libinferd_span.so in
// round 2 (VERDICT r01 "dead A/B code"): gemm_tiled256_kernel (8 waves, 256x256, double-
// buffered LDS) and gemm_ring256_kernel (8 waves, 10-slot LDS ring, look-ahead 8).  Both were
// measured slower than the 4-wave gemm_w4 / gemm_w4p bodies (ring 1173-1344 TF/s
// against 1250-1487 for w4p on the Qwen3-32B shapes).  Last built and tested in commit 2795314
// (inferd_amd/csrc/gemm.hip there); kept for the hazard derivation DESIGN.md cites.
// They need SplitTail / tile_order from inferd_amd/csrc/gemm.hip to compile.
#include "../../inferd_amd/csrc/common.h"
#include "../../inferd_amd/csrc/kernels.h"
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

