// Shared device helpers for the gfx950 (CDNA4) span kernels.
//
// Device data layouts (all bf16 unless stated):
//
//  * "Fragment-packed" weight W[N][K] (nn.Linear layout, N out-features, K in-features),
//    N % 16 == 0, K % 32 == 0.  Tile (nt, kt) covers rows 16*nt..+15 and columns
//    32*kt..+31 and is 1 KiB, stored at element offset (nt*KT + kt)*512.  Inside a tile,
//    lane l (0..63) owns 8 consecutive elements at offset l*8:
//        W[16*nt + (l & 15)][32*kt + 8*(l >> 4) + j],  j = 0..7
//    which is exactly the B operand of v_mfma_f32_16x16x32_bf16 for C = X * W^T, so a
//    wave fetches one whole tile with ONE global_load_dwordx4 (1 KiB contiguous).
//
//  * Paged KV cache: pool[layer][page][K|V][kv_head][64 tokens x 128 dims] with each
//    (page, K|V, kv_head) block 16 KiB.  Tiles are 1 KiB, 64 lanes x 8 elements:
//      K block: tile (tb, ks) at ((tb*4 + ks)*64 + l)*8 holds
//               K[token 16*tb + (l & 15)][dim 32*ks + 8*(l >> 4) + j]
//               (A operand of S^T = K * Q^T)
//      V block: tile (kt, db) at ((kt*8 + db)*64 + l)*8 holds
//               V[token 32*kt + vperm(l >> 4, j)][dim 16*db + (l & 15)]
//               vperm(g, j) = j < 4 ? 4g + j : 16 + 4g + (j - 4)
//               (A operand of O^T = V^T * P^T; the permutation matches the register
//               layout the S^T accumulators already have, so P needs no shuffles).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16;
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));

#define KV_PAGE 64          // tokens per KV page
#define HEAD_DIM 128        // Qwen3 head_dim (all sizes)
#define KV_BLOCK_ELEMS (KV_PAGE * HEAD_DIM)
// A layer's KV pool is laid out in super-pages of KV_SUPER pages:
//   [phys / 16][kv head][phys % 16][K | V][64 tokens x 128 dims]  (16 KiB per block)
// so a (sequence, kv head)'s consecutive pages are one contiguous run (up to 512 KiB): the
// decode attention's per-(sequence, head) read then streams like a flat read (22.7 vs 29.2
// us for Qwen3-8B B=16 ctx 2048, tools/attn_lab.hip).  Pools span a multiple of 16 pages.
#define KV_SUPER 16
__host__ __device__ __forceinline__ int64_t kv_block(int phys, int kind, int g, int KV) {
  return ((((int64_t)(phys / KV_SUPER) * KV + g) * KV_SUPER + (phys % KV_SUPER)) * 2 + kind) * KV_BLOCK_ELEMS;
}

__device__ __forceinline__ float bf2f(u16 b) { return __uint_as_float(((uint32_t)b) << 16); }
__device__ __forceinline__ u16 f2bf(float f) {
  __bf16 h = (__bf16)f;  // v_cvt_pk_bf16_f32, round-to-nearest-even
  return __builtin_bit_cast(u16, h);
}
// round an fp32 value to bf16 precision (models a torch bf16 op's output rounding)
__device__ __forceinline__ float rbf(float f) { return bf2f(f2bf(f)); }

__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ bf16x8 as_bf16x8(const u16x8& v) { return __builtin_bit_cast(bf16x8, v); }

__device__ __forceinline__ int vperm(int g, int j) { return j < 4 ? 4 * g + j : 16 + 4 * g + (j - 4); }

// Counted wait on this wave's vector-memory queue (loads, stores and LDS-DMA in issue
// order).  Inline asm: invisible to hipcc's own waitcnt pass, so it is never merged away.
template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// Workgroup barrier that does NOT drain vmcnt (__syncthreads() would wait for every
// in-flight global_load_lds); memory clobber + sched barriers pin LDS accesses around it.
__device__ __forceinline__ void raw_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// The lane index recomputed by the instruction that defines it (v_mbcnt, no input register),
// inside an asm volatile the compiler can neither hoist nor CSE: per-lane addresses derived from
// it are recomputed where they are used instead of being kept live (and spilled) across a
// register-heavy loop -- threadIdx.x itself is only an initial register that would have to live.
__device__ __forceinline__ int opaque_lane() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}

// Host+device splitmix64 (oracle/weightgen.py defines the same function).
__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// orderable key of a float (larger float -> larger unsigned)
__device__ __forceinline__ uint32_t float_key(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// Fragment-packed activations: the row-tile mt, k-tile kt fragment of a [rows][K] bf16 matrix
// is 1 KiB at element ((mt * K/32 + kt) * 64 + lane) * 8, lane l holding row 16 mt + l % 16,
// columns 32 kt + 8 (l / 16) .. + 7 -- the MFMA A operand, so a decode GEMV wave reads it with
// one contiguous 1 KiB load instead of sixteen 64-B row pieces (tools/mk_lab.hip: the
// row-major read costs the down GEMV ~1.5 us).  Element (row, col) of a row_len-wide matrix:
__device__ __forceinline__ int64_t packed_index(int row, int col, int64_t row_len) {
  return ((int64_t)(row >> 4) * (row_len >> 5) + (col >> 5)) * 512 + (row & 15) * 8 + ((col & 31) >> 3) * 128 +
         (col & 7);
}
