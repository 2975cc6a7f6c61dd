// Prefill attention, one wave per SIMD (gfx950, v_mfma_f32_32x32x16_bf16).
//
// Reference: Qwen3Attention.forward + SDPA / eager_attention_forward
// (models/qwen3/server/qwen3_server_module.py:126-162, :67-89) with the causal mask of
// petals/partitioned_models.py:28-35: fp32 scores, online softmax, P rounded to bf16 for P.V,
// O normalised in fp32 and rounded once (the same rounding points as attention.hip).
//
// Why this body.  The 2-waves-per-SIMD kernel (attention.hip attn_prefill_kernel) holds 32 query
// rows per wave with 16x16x32 MFMAs: every K/V fragment read from LDS feeds 2 MFMAs, so LDS reads
// plus the staging DMA take as many CU cycles as the matrix pipe, and each wave's
// S -> softmax -> P.V chain is latency-bound (49 % MFMA busy).  Here a workgroup of 4
// waves owns 256 query rows of one head, one wave per SIMD with the whole 512-register file:
//   AGPRs: O^T (4 dim blocks x 2 query blocks of 32x32 fp32 = 128), Q (64), the next page's K (64)
//   VGPRs: two score sets S (page i being normalised, page i+1 being accumulated), P, V fragments.
// Each 32x32x16 MFMA reads one fragment per 32 query rows, half the LDS traffic per flop, and
// leaves 24 of its 32 issue cycles to other instructions.  The page loop is software-pipelined
// by hand (cdna_hip_programming.md §B attention, one-wave-per-SIMD structure):
//   phase A_i : S_{i+1} = K_{i+1} Q^T (32 MFMAs)  ||  exp / row sums / bf16 packing of page i
//   phase B_i : O^T += V_i^T P_i^T   (32 MFMAs)  ||  rest of page i's softmax, row max of S_{i+1},
//                                                    LDS reads of V_i and K_{i+2}
// Each MFMA is followed by its fillers and a scheduling barrier, so hipcc keeps the placement;
// MFMAs, LDS reads and waits are inline asm (hipcc neither counts those reads nor pads MFMA
// hazards: every filler reads MFMA results >= 2 MFMA slots after they were written, P fragments
// are packed >= 1 slot before their MFMA, and the plain-code paths pad with s_nop).
//
// Layouts (common.h pages are fragment-ordered for 16x16x32 MFMAs; read here with per-lane
// permutations, conflict-free: every read is four contiguous 256-B runs):
//  * S^T = K Q^T, 32 tokens x 32 queries per tile: A = K (lane: token tau(l % 32), dims 8(l/32)..),
//    B = Q^T, C: lane = query l % 32, register g = S^T row (g&3) + 8(g>>2) + 4(l/32).
//    tau swaps rows 8-15 and 16-23, so registers 8s..8s+7 of a tile are exactly the P^T operand of
//    k-step s of the next product (cdna_hip_programming.md §3 "accumulator tile as operand") AND
//    index the tokens of one 16-byte chunk of the page's V tiles (quarter q = 2s + l/32).
//  * O^T = V^T P^T: A = V^T (lane: dim l % 32 of a 32-dim block, 8 tokens of quarter 2s + l/32),
//    B = P^T (bf16 pairs of S^T registers), C = O^T (lane = query, registers = dims).
// K/V pages are staged once per workgroup by LDS-DMA into a ring of four 32-KiB buffers, page i+3
// issued at the top of iteration i (after the one barrier per page).
#include <stdint.h>

#include <utility>

#include "../../inferd_amd/csrc/common.h"
#include "../../inferd_amd/csrc/kernels.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned u32x4v __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void* lds_ptr;
typedef const __attribute__((address_space(4))) int* cptr;

// AP_PROBE (lab builds only, tools/build_attn_probes.sh; wrong output, timing only): 1 no softmax
// fillers, 2 no per-page vmcnt wait/barrier, 3 no LDS reads in the phases, 4 no row-max chain;
// AP_NOWAIT: no lgkmcnt waits in the phases; AP_NODMA: no page staging after the prologue
#ifndef AP_PROBE
#define AP_PROBE 0
#endif
#ifndef AP_SORD
#define AP_SORD 1
#endif
// K fragment f of a page (the f-th used in phase A): AP_SORD 1 = c-major (f = 2c + tb: the four
// score tiles accumulate round-robin, each MFMA 4 slots after its predecessor on the same tile),
// 0 = tb-major (f = 8 tb + c: a tile's predecessor 2 slots back)
constexpr int frag_tb(int f) { return AP_SORD ? (f & 1) : (f >> 3); }
constexpr int frag_c(int f) { return AP_SORD ? (f >> 1) : (f & 7); }
constexpr int NA = 42;        // softmax values (of a lane's 64 per page) finished in phase A
constexpr float THR = 8.0f;   // lazy rescale threshold, log2 units (attention.hip RESCALE_THR)
constexpr int PAGE_BYTES = 32768;
constexpr int NBUF = 5;  // page j in buffer j % 5: DMA issued 4 pages (2 iterations of slack) ahead
// W64_CUTS (round 6): the round-4 VALU cuts of attention.hip in this body -- Q
// prescaled by scale*log2(e) once, the running -m on the first S MFMA's C operand (a per-query VGPR
// tuple, refreshed when m moves), so a score costs v_exp_f32 + a row-sum add + half a cvt_pk; the
// fillers are placed by tools/labsrc/w64_sched.py (<= 24 issue cycles per MFMA gap)
#ifndef W64_CUTS
#define W64_CUTS 0
#endif
#if W64_CUTS
#if W64_SCHED == 46
#include "w64_sched_dl46.h"
#else
#include "w64_sched.h"
#endif
#endif
#ifndef W64_LACC
#define W64_LACC 2
#endif
constexpr int LACC = W64_LACC;  // row-sum chains per query block

// ---- fixed schedule (global slot g: 0..31 phase A, 32..63 phase B) --------------------------
// softmax value v of a lane: tile tb = v >> 5, query block nq = (v >> 4) & 1, register v & 15
constexpr int fslot(int v) { return v < NA ? v * 32 / NA : 32 + (v - NA) / 2; }
// Phase A slot G: K fragment f = G / 2 (tb = f / 8, c = f % 8) times Q block nq = G % 2, so the tb = 0
// score tiles of page i+1 are accumulated in slots 0-15 and the tb = 1 tiles only from slot 16, when
// page i's tb = 0 tiles have been packed into P (fewer live registers).
// LDS reads of one iteration, at most one per slot, in issue order: K fragment f of
// page i+1 (f >= 3) at phase-A slot 2f - 6, three slots of MFMAs ahead of its first use (slot 2f);
// V(kk, db) of page i ahead of its P.V slice; K fragments 0..2 of page i+2 at the end of phase B
// (the next phase A starts on them).  K lives in a KR-fragment AGPR ring (fragment f in kr[f % KR]).
constexpr int kslot(int f) { return f >= 3 ? 2 * f - 6 : 49 + 2 * f; }  // f < 3: page i+2, early enough to land before phase B ends
// V(kk, db) four slots ahead of its first P.V MFMA (slot 32 + 8kk + 2db): three fragments live
constexpr int vslot(int kk, int db) { return 28 + 8 * kk + 2 * db; }
constexpr int KR = 6;  // K ring: fragment f in kr[f % KR], read 6 slots before use, its predecessor
                       // f - KR last used 5 slots before that read
constexpr int reads_in(int g) {
  int n = 0;
  for (int kk = 0; kk < 4; ++kk)
    for (int db = 0; db < 4; ++db) n += vslot(kk, db) == g;
  for (int f = 0; f < 16; ++f) n += kslot(f) == g;
  return n;
}
constexpr int reads_before(int g) {
  int n = 0;
  for (int x = 0; x < g; ++x) n += reads_in(x);
  return n;
}
// lgkmcnt before the MFMA of slot g that first consumes the read issued in slot rs: the reads
// issued after it (a slot's read follows its MFMA)
constexpr int rd_wait(int g, int rs) { return reads_before(g) - reads_before(rs) - 1; }
static_assert(reads_in(0) == 1 && reads_in(28) == 1 && reads_in(49) == 1 && reads_in(48) == 1, "one read per slot");
// byte offsets of the reads from the lane's base in a page buffer
constexpr int koff(int tb, int c) { return tb * 8192 + (c >> 1) * 1024 + (c & 1) * 512; }
constexpr int voff(int kk, int db) { return 16384 + (kk >> 1) * 8192 + db * 2048 + (kk & 1) * 512; }

__device__ __forceinline__ void mfma_s0(f32x16& d, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(d) : "a"(a), "a"(b));
}
__device__ __forceinline__ void mfma_sc(f32x16& d, const bf16x8& a, const bf16x8& b, const f32x16& c) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %3" : "=&v"(d) : "a"(a), "a"(b), "v"(c));
}
__device__ __forceinline__ void mfma_s(f32x16& d, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(d) : "a"(a), "a"(b));
}
__device__ __forceinline__ void mfma_o(f32x16& d, const bf16x8& a, const u32x4v& b) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(d) : "v"(a), "v"(b));
}
template <int OFF>
__device__ __forceinline__ void rd_a(bf16x8& d, unsigned addr) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=a"(d) : "v"(addr), "n"(OFF));
}
template <int OFF>
__device__ __forceinline__ void rd_v(bf16x8& d, unsigned addr) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(d) : "v"(addr), "n"(OFF));
}
#ifndef AP_NOWAIT
#define AP_NOWAIT 0
#endif
#ifndef AP_NODMA
#define AP_NODMA 0
#endif
#ifndef AP_STAMP
#define AP_STAMP 0  // lab: s_memtime stamps of block 0 / wave 0 per page (inferd_lab_stamps)
#endif
#if AP_STAMP
__device__ unsigned long long ap_stamps[8 * 160];
#endif
#ifndef AP_DMA_SAME
#define AP_DMA_SAME 0  // lab: every page staged from page 0 (L2-resident source, same LDS writes)
#endif
__device__ __forceinline__ void rd_b32(int& d, unsigned addr) {
  asm volatile("ds_read_b32 %0, %1" : "=v"(d) : "v"(addr));
}
template <int N>
__device__ __forceinline__ void lgkm_wait_i(int& pin) {
  asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(pin) : "n"(N));
}
template <int N>
__device__ __forceinline__ void lgkm_wait(bf16x8& pin) {
  if constexpr (AP_NOWAIT) asm volatile("" : "+v"(pin));
  else asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(pin) : "n"(N));
}
template <int N>
__device__ __forceinline__ void lgkm_wait_a(bf16x8& pin) {
  if constexpr (AP_NOWAIT) asm volatile("" : "+a"(pin));
  else asm volatile("s_waitcnt lgkmcnt(%1)" : "+a"(pin) : "n"(N));
}
__device__ __forceinline__ void lgkm_drain() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
// >= 16 wait states: an MFMA result read by plain code (hipcc does not see asm MFMAs)
__device__ __forceinline__ void mfma_drain() { asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory"); }
#define SLOT_END() __builtin_amdgcn_sched_barrier(0)
#define AI __attribute__((always_inline))

// in-place VALU on score-tile elements as inline asm: C++ element updates of an f32x16 made hipcc
// rebuild whole 16-register tuples (copies and spills); asm "+v" on an element edits it in place.
// Hazards are the caller's: an exp result is read >= 1 instruction later (trans forwarding), a
// permlane source is written >= 2 states earlier (the s_nop inside).
// (macros: a vector element cannot bind to a reference parameter)
#define A_FMA(x, c, mneg) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x) : "v"(c), "v"(mneg))
#define A_EXP(x) asm volatile("v_exp_f32 %0, %0" : "+v"(x))
#define A_ADD(acc, x) asm volatile("v_add_f32 %0, %0, %1" : "+v"(acc) : "v"(x))
#define A_CVT(d, lo, hi) asm volatile("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(d) : "v"(lo), "v"(hi))
#define A_MAX3(d, a, b, c) asm volatile("v_max3_f32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c))
#define A_MAX(d, a, b) asm volatile("v_max_f32 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b))
// element := -inf where limit < k (k a per-element constant): v_bfi on an all-ones sign mask
#define A_MASK(x, limit, k)                                                                                 \
  do {                                                                                                      \
    int msk_;                                                                                               \
    asm volatile("v_subrev_u32 %0, %2, %1\n\tv_ashrrev_i32 %0, 31, %0\n\ts_nop 0\n\tv_bfi_b32 %0, %0, %3, %4" \
                 : "=&v"(msk_) : "v"(limit), "v"(k), "v"(0xff800000u), "v"(x));                            \
    asm volatile("v_mov_b32 %0, %1" : "=v"(x) : "v"(msk_));                                                 \
  } while (0)

__device__ __forceinline__ unsigned pack_bf16(float a, float b) {
  const bf16x2 t = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(unsigned, t);
}

// S^T row of register g in lane half h, and the page-relative token it holds (tau)
__device__ __forceinline__ int srow(int g, int h) { return (g & 3) + 8 * (g >> 2) + 4 * h; }
__device__ __forceinline__ int tau(int r) { return (r >= 8 && r < 16) ? r + 8 : (r >= 16 && r < 24) ? r - 8 : r; }

}  // namespace

// grid (ceil(max_q_len / 256) * H, B), 256 threads, dynamic LDS NBUF * 32 KiB
__global__ __launch_bounds__(256, 1) void attn_prefill_w64_kernel(const u16* __restrict__ q, const u16* __restrict__ kv,
                                                                  AttnBatch b, int H, int KV, float cl,
                                                                  u16* __restrict__ out, int order) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int bseq = blockIdx.y;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int swave = __builtin_amdgcn_readfirstlane(wave);
  const int r = lane & 31, hh = lane >> 5;
  const int n_rep = H / KV;
  const int mqb = (b.max_q_len + 255) / 256;
  int h, qbi;
  if (order == 1) {  // XCD-grouped: a GQA group's heads adjacent on one XCD (attention.hip)
    const int n = gridDim.x, x = blockIdx.x;
    const int wg = (x & 7) * (n >> 3) + (x >> 3);
    const int rr = wg % n_rep, t = wg / n_rep;
    qbi = t % mqb;
    h = (t / mqb) * n_rep + rr;
  } else {
    h = blockIdx.x / mqb;
    qbi = blockIdx.x % mqb;
  }
  const int g = h / n_rep;
  const int t0 = b.seq_start[bseq];
  const int T = b.seq_start[bseq + 1] - t0;
  const int nqb = (T + 255) / 256;
  const int qb = mqb - 1 - qbi;  // heaviest first
  if (qb >= nqb) return;
  const int qb0 = qb * 256;
  const int wrow0 = qb0 + swave * 64;

  // ---- this lane's two query rows (one per 32-row block), their positions and Q fragments
  int lim[2], tokrow[2];
  bool valid[2];
  bf16x8 qf[2][8];
#pragma unroll
  for (int nq = 0; nq < 2; ++nq) {
    const int row = wrow0 + nq * 32 + r;
    valid[nq] = row < T;
    tokrow[nq] = t0 + (valid[nq] ? row : T - 1);
    lim[nq] = b.positions[tokrow[nq]];
    const u16* qp = q + ((int64_t)tokrow[nq] * H + h) * HEAD_DIM + 8 * hh;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      qf[nq][c] = *(const bf16x8*)(qp + c * 16);
#if W64_CUTS
#pragma unroll
      for (int j = 0; j < 8; ++j) qf[nq][c][j] = (__bf16)((float)qf[nq][c][j] * cl);
#endif
    }
  }
#pragma unroll
  for (int nq = 0; nq < 2; ++nq)
#pragma unroll
    for (int c = 0; c < 8; ++c) asm volatile("" : "+a"(qf[nq][c]));  // Q lives in AGPRs
  const int wg_last = b.positions[t0 + min(qb0 + 255, T - 1)];
  const int n_pages = wg_last / KV_PAGE + 1;
  // the wave's pages: up to its last row's position; masks on pages reaching past its first row
  const bool wave_live = wrow0 < T;
  const int wave_last_page = wave_live ? b.positions[t0 + min(wrow0 + 63, T - 1)] / KV_PAGE : -1;
  const int wave_min_lim = wave_live ? b.positions[t0 + wrow0] : 0;

  // ---- K/V staging: 8 x 1 KiB LDS-DMA pieces per wave per page (common.h page = K 16 KiB | V 16 KiB)
  const cptr bt = (cptr)(b.block_table + (int64_t)bseq * b.max_pages);
  // phys: the page's block-table entry (the loop reads it one page ahead, so the scalar load's
  // latency is not waited for in front of the DMA issue)
  auto stage_half = [&](int page, int phys, int half) AI {
    const __amdgpu_buffer_rsrc_t pg =
        __builtin_amdgcn_make_buffer_rsrc((void*)(kv + kv_block(phys, 0, g, KV)), 0, 2 * KV_BLOCK_ELEMS * 2, 0x00020000);
    char* base = lds + (page % NBUF) * PAGE_BYTES;
#pragma unroll
    for (int pc = 4 * half; pc < 4 * half + 4; ++pc) {
      const int piece = swave * 8 + pc;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(pg, (lds_ptr)(base + piece * 1024), 16, lane * 16, piece * 1024, 0, 0);
    }
  };
  auto stage = [&](int page, int phys) AI {
    stage_half(page, phys, 0);
    stage_half(page, phys, 1);
  };
  // this wave's DMA of page i+2 (issued an iteration ago) has landed; the page barrier
  auto page_barrier = [&](int i) AI {
    if constexpr (AP_PROBE != 2) asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  };
  // per-lane read bases (LDS byte addresses) within a page buffer
  const unsigned lds0 = (unsigned)(uintptr_t)(lds_ptr)lds;
  const int tk = tau(r);
  const unsigned lane_k = (tk >> 4) * 4096 + ((tk & 15) + 16 * hh) * 16;
  const unsigned lane_v = (r >> 4) * 1024 + ((r & 15) + 16 * hh) * 16;
  // buffer offsets as wave-uniform scalars (a % 5 left to hipcc spread VGPR address variants and spilled)
  auto boff = [&](int page) AI { return (unsigned)__builtin_amdgcn_readfirstlane((unsigned)(page % NBUF) * PAGE_BYTES); };
  auto kbase = [&](int page) AI { return lds0 + boff(page) + lane_k; };
  auto vbase = [&](int page) AI { return lds0 + boff(page) + lane_v; };

  f32x16 s[2][2][2];  // [set][nq][tb]
  f32x16 o[4][2];     // O^T [dim block][nq]
#pragma unroll
  for (int db = 0; db < 4; ++db)
#pragma unroll
    for (int nq = 0; nq < 2; ++nq) {
      o[db][nq] = f32x16{};
      asm volatile("" : "+a"(o[db][nq]));
    }
  bf16x8 kr[KR];  // K fragment ring (AGPRs)
  bf16x8 vf[4][4];
  float lacc[2][LACC];
#pragma unroll
  for (int j = 0; j < LACC; ++j) lacc[0][j] = lacc[1][j] = 0.f;
#if W64_CUTS
  f32x16 mc[2];  // -m per query row, the C operand of each score tile's first MFMA
#endif
  float m[2] = {-INFINITY, -INFINITY}, mnew[2] = {-INFINITY, -INFINITY};
  bool pend = false;

  // causal mask of a score set holding page p (plain code, >= 16 wait states after its MFMAs).
  // Register gi of lane half hh holds token p*64 + tb*32 + tau(srow(gi, 0)) + 4hh (tau moves
  // whole 8-row blocks), so each element compares a constant with one per-lane bound.
  auto mask_set = [&](f32x16 (&ss)[2][2], int p) AI {
#pragma unroll
    for (int nq = 0; nq < 2; ++nq) {
      const int L = lim[nq] - p * KV_PAGE - 4 * hh;
#pragma unroll
      for (int tb = 0; tb < 2; ++tb)
#pragma unroll
        for (int gi = 0; gi < 16; ++gi) A_MASK(ss[nq][tb][gi], L, tb * 32 + tau(srow(gi, 0)));
    }
  };
  // row max of a score set (log2 units) -> mnew, pend (plain code)
  auto max_set = [&](f32x16 (&ss)[2][2]) AI {
#pragma unroll
    for (int nq = 0; nq < 2; ++nq) {
      float a = -INFINITY;
#pragma unroll
      for (int tb = 0; tb < 2; ++tb)
#pragma unroll
        for (int gi = 0; gi < 16; ++gi) a = fmaxf(a, ss[nq][tb][gi]);
      const unsigned u = __float_as_uint(a);
      const auto sw = __builtin_amdgcn_permlane32_swap(u, u, false, false);
      a = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
      mnew[nq] = fmaxf(m[nq], W64_CUTS ? a : a * cl);
    }
    pend = __builtin_amdgcn_ballot_w64(mnew[0] > m[0] + THR || mnew[1] > m[1] + THR) != 0;
  };
#if W64_CUTS
  // the C tuples from m (plain code; the s_nop covers VALU write -> MFMA SrcC read)
  auto set_mc = [&]() AI {
#pragma unroll
    for (int nq = 0; nq < 2; ++nq)
#pragma unroll
      for (int j = 0; j < 16; ++j) mc[nq][j] = -m[nq];
    asm volatile("s_nop 4" ::: "memory");
  };
  // a score set computed against one m moved to another: x += delta[nq]
  auto shift_set = [&](f32x16 (&ss)[2][2], float d0, float d1) AI {
#pragma unroll
    for (int nq = 0; nq < 2; ++nq) {
      const float dl = nq ? d1 : d0;
#pragma unroll
      for (int tb = 0; tb < 2; ++tb)
        [&]<int... R>(std::integer_sequence<int, R...>) AI {
          ([&]() AI {
            constexpr int rr = R;
            f32x16& x = ss[nq][tb];
            const float dd = dl;  // named: a variable used only inside an asm operand is not captured
            A_ADD(x[rr], dd);
          }(), ...);
        }(std::make_integer_sequence<int, 16>{});
    }
  };
#endif
  // apply a pending rescale (O, l at the old max -> new max): plain code, rare
  auto rescale = [&]<int CUR>() AI {
    if (!pend) return;
    mfma_drain();
#if W64_CUTS
    // page i's scores were taken against the old m: move them with O and l
    shift_set(s[CUR], m[0] - mnew[0], m[1] - mnew[1]);
#endif
#pragma unroll
    for (int nq = 0; nq < 2; ++nq) {
      const float alpha = (m[nq] == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(m[nq] - mnew[nq]);
#pragma unroll
      for (int j = 0; j < LACC; ++j) lacc[nq][j] *= alpha;
#pragma unroll
      for (int db = 0; db < 4; ++db) o[db][nq] *= alpha;
      m[nq] = mnew[nq];
    }
#if W64_CUTS
    set_mc();
#endif
    asm volatile("s_nop 4" ::: "memory");
    pend = false;
  };

  // ---- softmax stream fillers on the set holding page i (slot G): F = scale and subtract the
  // max, E = exp2, ADD = row sums (two chains per query block), CVT = bf16 pair into P
  float mneg[2];
  auto soft = [&]<int G, int CUR>(u32x4v (&pf)[2][4]) AI {
    if constexpr (AP_PROBE == 1) return;
    [&]<int... V>(std::integer_sequence<int, V...>) AI {
      (
          [&]() AI {
            constexpr int tb = V >> 5, nq = (V >> 4) & 1, reg = V & 15;
            // named references: a variable used only inside an asm operand is not captured
            f32x16& x = s[CUR][nq][tb];
            u32x4v& pw = pf[nq][tb * 2 + (reg >> 3)];
            float& la = lacc[nq][reg % LACC];
#if W64_CUTS
            if constexpr (EXP_SLOT[V] == G) A_EXP(x[reg]);
            if constexpr (ADD_SLOT[V] == G) A_ADD(la, x[reg]);
            if constexpr ((V & 1) == 0 && CVT_SLOT[V] == G) A_CVT(pw[(reg & 7) >> 1], x[reg], x[reg + 1]);
#else
            const float mn = mneg[nq], c2 = cl;
            if constexpr (fslot(V) == G) A_FMA(x[reg], c2, mn);
            if constexpr (fslot(V) + 1 == G) A_EXP(x[reg]);
            if constexpr (fslot(V) + 2 == G) A_ADD(la, x[reg]);
            if constexpr ((V & 1) == 0 && fslot(V + 1) + 3 == G) A_CVT(pw[(reg & 7) >> 1], x[reg], x[reg + 1]);
#endif
          }(),
          ...);
    }(std::make_integer_sequence<int, 64>{});
  };
  // ---- phase A_i: S_{i+1} MFMAs || softmax of page i || K_{i+1} and V_i slice-0 reads
  auto phase_a = [&]<int CUR, bool NEXT>(int page, u32x4v (&pf)[2][4]) AI {
    constexpr int NXT = CUR ^ 1;
    mneg[0] = -m[0];
    mneg[1] = -m[1];
    const unsigned va = vbase(page), ka = kbase(page + 1);
    [&]<int... G>(std::integer_sequence<int, G...>) AI {
      (
          [&]() AI {
            constexpr int f = G >> 1, tb = frag_tb(f), c = frag_c(f), nq = G & 1;
            if constexpr (NEXT) {
              if constexpr (f >= 3 && (G & 1) == 0) lgkm_wait_a<rd_wait(G, kslot(f))>(kr[f % KR]);
              if constexpr (c == 0 && W64_CUTS)
                mfma_sc(s[NXT][nq][tb], kr[f % KR], qf[nq][c], mc[nq]);
              else if constexpr (c == 0)
                mfma_s0(s[NXT][nq][tb], kr[f % KR], qf[nq][c]);
              else
                mfma_s(s[NXT][nq][tb], kr[f % KR], qf[nq][c]);
            }
            soft.template operator()<G, CUR>(pf);
            if constexpr (AP_PROBE != 3 && NEXT && (G & 1) == 0 && G <= 24) {
              constexpr int fr = G / 2 + 3;
              rd_a<koff(frag_tb(fr), frag_c(fr))>(kr[fr % KR], ka);
            }
            if constexpr (AP_PROBE != 3 && G >= 28 && (G & 1) == 0) rd_v<voff(0, (G - 28) / 2)>(vf[0][(G - 28) / 2], va);
            SLOT_END();
          }(),
          ...);
    }(std::make_integer_sequence<int, 32>{});
  };
  // ---- phase B_i: P_i V_i MFMAs || softmax tail of page i || row max of S_{i+1} || V_i, K_{i+2} reads
  auto phase_b = [&]<int CUR, bool NEXT>(int page, u32x4v (&pf)[2][4]) AI {
    constexpr int NXT = CUR ^ 1;
    const unsigned va = vbase(page), ka = kbase(page + 2);
    float mx[2][2];
    [&]<int... K>(std::integer_sequence<int, K...>) AI {
      (
          [&]() AI {
            constexpr int G = 32 + K;
            constexpr int kk = K >> 3, db = (K >> 1) & 3, nq = K & 1;
            if constexpr ((K & 1) == 0) lgkm_wait<rd_wait(G, vslot(kk, db))>(vf[kk][db]);
            mfma_o(o[db][nq], vf[kk][db], pf[nq][kk]);
            soft.template operator()<G, CUR>(pf);
            // row max of S_{i+1}: chains (nq, tb), 8 max3 steps each, slots 44..59
            [&]<int... C>(std::integer_sequence<int, C...>) AI {
              (
                  [&]() AI {
                    constexpr int ch = C, cnq = ch >> 1, ctb = ch & 1;
#if W64_CUTS
                    // MAX_SLOT[ch][t] == G for at most one t per chain and slot (the schedule keeps a
                    // chain's steps in separate slots, so the step index is found by search)
                    constexpr int t = [] {
                      for (int u = 0; u < 8; ++u)
                        if (MAX_SLOT[ch][u] == G) return u;
                      return -1;
                    }();
                    if constexpr (AP_PROBE != 4 && NEXT && t >= 0) {
#else
                    constexpr int t = (G - 44 - (ch >> 1)) / 2;
                    if constexpr (AP_PROBE != 4 && NEXT && G >= 44 && G < 60 && ((G - 44) & 1) == (ch >> 1) && t >= 0 && t < 8) {
#endif
                      f32x16& x = s[NXT][cnq][ctb];
                      float& mc = mx[cnq][ctb];
                      if constexpr (t == 0)
                        A_MAX3(mc, x[0], x[1], x[2]);
                      else if constexpr (t < 7)
                        A_MAX3(mc, mc, x[2 * t + 1], x[2 * t + 2]);
                      else
                        A_MAX(mc, mc, x[15]);
                    }
                  }(),
                  ...);
            }(std::make_integer_sequence<int, 4>{});
            if constexpr (NEXT && (G == 60 || G == 61)) {
              constexpr int cnq = G - 60;
              float a = fmaxf(mx[cnq][0], mx[cnq][1]);
              const unsigned u = __float_as_uint(a);
              const auto sw = __builtin_amdgcn_permlane32_swap(u, u, false, false);
              a = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
              mnew[cnq] = W64_CUTS ? m[cnq] + fmaxf(a, 0.f) : fmaxf(m[cnq], a * cl);
            }
#if W64_CUTS
            // the next phase A's C tuples (-m; a rescale in between sets them again)
            [&]<int... J>(std::integer_sequence<int, J...>) AI {
              (
                  [&]() AI {
                    if constexpr (MOV_SLOT[J] == G) {
                      f32x16& t = mc[J >> 4];
                      if constexpr ((J & 15) == 0) {  // the tuple's old value is dead from here
                        f32x16 dead;
                        t = dead;
                      }
                      const float mn = -m[J >> 4];
                      asm volatile("v_mov_b32 %0, %1" : "=v"(t[J & 15]) : "v"(mn));
                    }
                  }(),
                  ...);
            }(std::make_integer_sequence<int, 32>{});
#endif
            if constexpr (NEXT && G == 62) pend = __builtin_amdgcn_ballot_w64(mnew[0] > m[0] + THR || mnew[1] > m[1] + THR) != 0;
            // LDS reads (a slot's V read before its K read)
            [&]<int... R>(std::integer_sequence<int, R...>) AI {
              (
                  [&]() AI {
                    constexpr int rk = R >> 2, rd = R & 3;
                    if constexpr (AP_PROBE != 3 && vslot(rk, rd) == G) rd_v<voff(rk, rd)>(vf[rk][rd], va);
                  }(),
                  ...);
            }(std::make_integer_sequence<int, 16>{});
            [&]<int... F>(std::integer_sequence<int, F...>) AI {
              ((AP_PROBE != 3 && NEXT && kslot(F) == G ? rd_a<koff(frag_tb(F), frag_c(F))>(kr[F], ka) : void()), ...);
            }(std::make_integer_sequence<int, 3>{});
            SLOT_END();
          }(),
          ...);
    }(std::make_integer_sequence<int, 32>{});
    lgkm_drain();
  };
  // S of one page, plain (prologue): K fragments through the ring in quarters, 32 MFMAs
  auto s_quarter = [&]<int SET, int QF>(unsigned ka) AI {
    [&]<int... I>(std::integer_sequence<int, I...>) AI {
      (rd_a<koff(frag_tb(4 * QF + I), frag_c(4 * QF + I))>(kr[I], ka), ...);
    }(std::make_integer_sequence<int, 4>{});
    lgkm_drain();
#pragma unroll
    for (int f = 0; f < 4; ++f)
#pragma unroll
      for (int nq = 0; nq < 2; ++nq) {
        const int c = frag_c(4 * QF + f), tb = frag_tb(4 * QF + f);
        if (c == 0)
          mfma_s0(s[SET][nq][tb], kr[f], qf[nq][c]);
        else
          mfma_s(s[SET][nq][tb], kr[f], qf[nq][c]);
      }
  };
  auto s_page = [&]<int SET>(int page) AI {
    s_quarter.template operator()<SET, 0>(kbase(page));
    s_quarter.template operator()<SET, 1>(kbase(page));
    s_quarter.template operator()<SET, 2>(kbase(page));
    s_quarter.template operator()<SET, 3>(kbase(page));
  };
  // the first three K fragments of a page (the rest are read inside phase A)
  auto read_k = [&](int page) AI {
    const unsigned ka = kbase(page);
    rd_a<koff(frag_tb(0), frag_c(0))>(kr[0], ka);
    rd_a<koff(frag_tb(1), frag_c(1))>(kr[1], ka);
    rd_a<koff(frag_tb(2), frag_c(2))>(kr[2], ka);
    lgkm_drain();
  };

  // ---- prologue: pages 0..3 in flight, S_0, its max, K_1.  Iteration i issues DMA(i+4) (8 pieces
  // per wave), so at the top of iteration i+1, vmcnt(8) leaves only that one in flight: DMA(i+3),
  // needed from phase B_{i+1} on, has landed.  Block-table entries by scalar loads one iteration
  // ahead, alternating between two variables (one per half of the two-iteration loop body: no
  // register rotation, so hipcc waits for the load only where the next iteration uses it; a single
  // rotated variable made it wait in front of the DMA)
  int physv[2] = {0, 0};
  stage(0, bt[0]);
  if (n_pages > 1) stage(1, bt[1]);
  if (n_pages > 2) stage(2, bt[2]);
  if (n_pages > 3) stage(3, bt[3]);
  if (n_pages > 4) physv[0] = bt[4];
  if (n_pages > 3)
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // pages 0 and 1 landed (this wave's pieces)
  else
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  asm volatile("s_barrier" ::: "memory");
  if (wave_last_page >= 0) {
    s_page.template operator()<0>(0);
    mfma_drain();
    if (KV_PAGE - 1 > wave_min_lim) mask_set(s[0], 0);
    max_set(s[0]);
    m[0] = mnew[0];
    m[1] = mnew[1];
    pend = false;
#if W64_CUTS
    shift_set(s[0], -m[0], -m[1]);
    set_mc();
#endif
    if (wave_last_page >= 1) read_k(1);
  }

  // ---- page loop: iteration i multiplies page i; two iterations per trip (score sets swap)
  auto stamp = [&](int i, int k) AI {
#if AP_STAMP
    if (blockIdx.x == 0 && blockIdx.y == 0 && swave == 0 && lane == 0 && i < 160) {
      unsigned long long t;
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t));
      ap_stamps[i * 8 + k] = t;
    }
#endif
  };
  auto iter = [&]<int CUR>(int i) AI {
    stamp(i, 0);
    // page i+2 landed (this wave's pieces, issued two iterations ago) and every wave is done with
    // page i-1's buffer: refill it with page i+4
    if constexpr (AP_PROBE != 2) {
      if (i + 3 < n_pages)
        asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    }
    if (!AP_NODMA && i + 4 < n_pages) {
      stage(i + 4, physv[CUR]);
      // issued after the use of the previous one: SMEM returns out of order, so waiting for the old
      // entry would wait for the new load too
      if (i + 5 < n_pages) physv[CUR ^ 1] = bt[i + 5];
    }
    stamp(i, 1);
    if (i > wave_last_page) return;
    rescale.template operator()<CUR>();
    stamp(i, 2);
    // one code path for every page (a second register assignment for the wave's last page made
    // hipcc shuffle O between AGPR homes): on the last page the S_{i+1} slots score whatever the
    // next buffer holds and the mask turns all of it into -inf (its tokens lie past every row)
    u32x4v pf[2][4];  // P of page i: a fresh value per page (no false dependence on the last page's)
    phase_a.template operator()<CUR, true>(i, pf);
    stamp(i, 3);
    if ((i + 1) * KV_PAGE + KV_PAGE - 1 > wave_min_lim) {
      mfma_drain();
      mask_set(s[CUR ^ 1], i + 1);
    }
    stamp(i, 4);
    phase_b.template operator()<CUR, true>(i, pf);
    stamp(i, 5);
  };
  for (int i = 0; i < n_pages; i += 2) {
    iter.template operator()<0>(i);
    if (i + 1 < n_pages) iter.template operator()<1>(i + 1);
  }
  if (!wave_live) return;

  // ---- epilogue: l over both lane halves, O^T / l -> bf16 rows
  mfma_drain();
#pragma unroll
  for (int nq = 0; nq < 2; ++nq) {
    float l = lacc[nq][0];
#pragma unroll
    for (int j = 1; j < LACC; ++j) l += lacc[nq][j];
    const unsigned u = __float_as_uint(l);
    const auto sw = __builtin_amdgcn_permlane32_swap(u, u, false, false);
    l = __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
    const float inv = 1.0f / l;
    if (!valid[nq]) continue;
    u16* op = out + (int64_t)tokrow[nq] * H * HEAD_DIM + h * HEAD_DIM + 4 * hh;
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
      for (int G4 = 0; G4 < 4; ++G4) {
        u16x4 v;
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = f2bf(o[db][nq][4 * G4 + j] * inv);
        *(u16x4*)(op + db * 32 + 8 * G4) = v;
      }
  }
}

#if AP_STAMP
extern "C" int inferd_lab_stamps(unsigned long long* host) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(ap_stamps), sizeof(ap_stamps), 0, hipMemcpyDeviceToHost);
}
#endif

static bool w64_lds_ok() {
  static int ok = -1;
  if (ok < 0)
    ok = hipFuncSetAttribute((const void*)attn_prefill_w64_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                             NBUF * PAGE_BYTES) == hipSuccess;
  return ok == 1;
}

bool launch_attn_prefill_w64(const u16* q, const u16* kv_layer, const AttnBatch& b, int H, int KV, float scale,
                             u16* out, hipStream_t s) {
  if (!w64_lds_ok()) return false;
  const int n = (b.max_q_len + 255) / 256 * H;
  const int order = n % 8 == 0 ? 1 : 0;
  hipLaunchKernelGGL(attn_prefill_w64_kernel, dim3(n, b.B), dim3(256), NBUF * PAGE_BYTES, s, q, kv_layer, b, H, KV,
                     scale * 1.4426950408889634f, out, (order == 1 && n % 8 == 0) ? 1 : 0);
  return true;
}
