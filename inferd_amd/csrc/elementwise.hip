// Memory-bound per-token kernels of the Qwen3 span: weight generation / packing,
// RMSNorm, fused QK-norm + RoPE + paged KV write, embedding gather, rope table,
// final-norm gather and greedy-token decode.
//
// Reference semantics (file:line in /root/reference):
//   Qwen3RMSNorm.forward            models/qwen3/server/qwen3_server_module.py:19-25
//   q_norm/k_norm before RoPE       qwen3_server_module.py:134-142
//   rotate_half/apply_rotary        qwen3_server_module.py:43-54
//   DynamicCache.update (K/V append) qwen3_server_module.py:144-148
//   embed (first span)              petals/partitioned_models.py:48
//   final norm + greedy argmax      petals/partitioned_models.py:95-96,162
// Every bf16 rounding point of the reference's eager bf16 ops is reproduced (rbf()).
#include "common.h"
#include "kernels.h"

// ------------------------------------------------------------------ weight generation
__global__ void weightgen_kernel(u16* __restrict__ dst, int64_t n, uint64_t key, float scale,
                                 float center) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) {
    uint64_t z = splitmix64(key + (uint64_t)i);
    float t = (float)(uint32_t)(z >> 40) * 1.1920928955078125e-07f - 1.0f;  // exact
    float w = __fadd_rn(__fmul_rn(t, scale), center);                         // no FMA
    dst[i] = f2bf(w);
  }
}

void launch_weightgen(u16* dst, int64_t n, uint64_t key, float scale, float center, hipStream_t s) {
  int64_t blocks = (n + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(weightgen_kernel, dim3((unsigned)blocks), dim3(256), 0, s, dst, n, key, scale,
                     center);
}

// ------------------------------------------------------------------ fragment packing
// one thread per 16-byte chunk: chunk c = (nt*KT + kt)*64 + lane
__global__ void pack_kernel(const u16* __restrict__ src, int64_t ld, int N, int K, u16* __restrict__ dst) {
  int KT = K / 32;
  int64_t nchunks = (int64_t)(N / 16) * KT * 64;
  int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (; c < nchunks; c += stride) {
    int lane = (int)(c & 63);
    int64_t tile = c >> 6;
    int kt = (int)(tile % KT);
    int64_t nt = tile / KT;
    int64_t row = nt * 16 + (lane & 15);
    int col = kt * 32 + 8 * (lane >> 4);
    *(u16x8*)(dst + c * 8) = *(const u16x8*)(src + row * ld + col);
  }
}

void launch_pack(const u16* src, int64_t ld, int N, int K, u16* dst, hipStream_t s) {
  int64_t nchunks = (int64_t)(N / 16) * (K / 32) * 64;
  int64_t blocks = (nchunks + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(pack_kernel, dim3((unsigned)blocks), dim3(256), 0, s, src, ld, N, K, dst);
}

// inverse (tests / debugging): packed -> row-major
__global__ void unpack_kernel(const u16* __restrict__ src, int N, int K, u16* __restrict__ dst) {
  int KT = K / 32;
  int64_t nchunks = (int64_t)(N / 16) * KT * 64;
  int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (; c < nchunks; c += stride) {
    int lane = (int)(c & 63);
    int64_t tile = c >> 6;
    int kt = (int)(tile % KT);
    int64_t nt = tile / KT;
    int64_t row = nt * 16 + (lane & 15);
    int col = kt * 32 + 8 * (lane >> 4);
    *(u16x8*)(dst + row * K + col) = *(const u16x8*)(src + c * 8);
  }
}

void launch_unpack(const u16* src, int N, int K, u16* dst, hipStream_t s) {
  int64_t nchunks = (int64_t)(N / 16) * (K / 32) * 64;
  int64_t blocks = (nchunks + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(unpack_kernel, dim3((unsigned)blocks), dim3(256), 0, s, src, N, K, dst);
}

// ------------------------------------------------------------------ decode-step advance
// Device-side scheduler step for a captured decode graph: the new token of sequence b sits
// at position ctx_lens[b] (the cached length), writes its K/V to the slot the block table
// gives for that position, and the cached length grows by one.  Runs in the graph's first
// node (decode_advance_kernel, or the first RMSNorm launch: NormPrologue), so a replay needs
// no host work.  A sequence whose block table is full gets slot -1 (no cache write) and sets
// err bit 2.
__device__ __forceinline__ void decode_advance_one(int32_t* positions, int32_t* slots, int32_t* ctx_lens,
                                                   const int32_t* block_table, int max_pages, int b, int32_t* err) {
  int p = ctx_lens[b];
  positions[b] = p;
  if (p / KV_PAGE < max_pages) {
    slots[b] = block_table[(int64_t)b * max_pages + p / KV_PAGE] * KV_PAGE + p % KV_PAGE;
    ctx_lens[b] = p + 1;
  } else {
    slots[b] = -1;
    atomicOr(err, 2);
  }
}

// A decode step's prologue where the span's first launch is not an RMSNorm (a span starting at
// an o projection): workgroup 0 runs the graph's scheduler step (NormPrologue positions), and
// workgroup r < M zeroes row r's words of the SSQ slots the span's decode GEMVs will fill.
__global__ __launch_bounds__(64) void step_prologue_kernel(unsigned long long* __restrict__ zero_slots,
                                                           int n_slots, NormPrologue pro) {
  const int row = blockIdx.x;
  if (pro.positions && row == 0)
    for (int b = threadIdx.x; b < pro.B; b += 64) decode_advance_one(pro.positions, pro.slots, pro.ctx_lens,
                                                                      pro.block_table, pro.max_pages, b, pro.err);
  for (int i = threadIdx.x; i < n_slots * SSQ_SHARDS * 2; i += 64) zero_slots[(int64_t)i * 64 + row] = 0ull;
}

void launch_step_prologue(unsigned long long* zero_slots, int n_slots, int M, const NormPrologue* pro_in,
                          hipStream_t s) {
  if (!zero_slots || M > 64) n_slots = 0;
  const NormPrologue pro = pro_in ? *pro_in : NormPrologue{};
  hipLaunchKernelGGL(step_prologue_kernel, dim3(M < 1 ? 1 : (M > 64 ? 1 : M)), dim3(64), 0, s, zero_slots, n_slots,
                     pro);
}

// ------------------------------------------------------------------ RMSNorm
// y = w * bf16(x * 1/sqrt(mean(x^2) + eps))     (qwen3_server_module.py:19-25)
// One 256-thread block per row; each thread keeps <= CH 8-element chunks in registers.
// If row_index != nullptr the block reads row row_index[blockIdx.x] (final-norm gather).
template <int CH>
__global__ __launch_bounds__(256) void rmsnorm_kernel(const u16* __restrict__ x, int64_t ldx,
                                                      const int32_t* __restrict__ row_index,
                                                      int row_sub, const u16* __restrict__ w,
                                                      u16* __restrict__ y, int64_t ldy, int N,
                                                      float eps, int pack, unsigned long long* zero_slots,
                                                      int n_slots, NormPrologue pro) {
  __shared__ float red[4];
  int row = blockIdx.x;
  if (pro.positions && row == 0)
    for (int b = threadIdx.x; b < pro.B; b += 256) decode_advance_one(pro.positions, pro.slots, pro.ctx_lens,
                                                                       pro.block_table, pro.max_pages, b, pro.err);
  // this row's words of the SSQ slots the span's decode GEMVs will fill (kernels.h DecodeNorm)
  for (int i = threadIdx.x; i < n_slots * SSQ_SHARDS * 2; i += 256) zero_slots[(int64_t)i * 64 + row] = 0ull;
  int src_row = row_index ? row_index[row] - row_sub : row;
  const u16* xr = x + (int64_t)src_row * ldx;
  if (pro.ids) {  // embedding gather (embed_kernel's checks)
    int id = pro.ids[row];
    if (id < 0 || id >= pro.vocab) {
      if (threadIdx.x == 0) atomicOr(pro.err, 1);
      id = 0;
    }
    xr = pro.table + (int64_t)id * N;
  }
  int nch = N / 8;
  float v[CH][8];
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    int ci = threadIdx.x + c * 256;
    if (ci < nch) {
      u16x8 p = *(const u16x8*)(xr + ci * 8);
      if (pro.x_out) *(u16x8*)(pro.x_out + (int64_t)row * N + ci * 8) = p;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v[c][j] = bf2f(p[j]);
        ss += v[c][j] * v[c][j];
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
  __syncthreads();
  ss = red[0] + red[1] + red[2] + red[3];
  float inv = 1.0f / sqrtf(ss / (float)N + eps);
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    int ci = threadIdx.x + c * 256;
    if (ci < nch) {
      u16x8 wp = *(const u16x8*)(w + ci * 8);
      u16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f2bf(bf2f(wp[j]) * rbf(v[c][j] * inv));
      // pack: y fragment-packed (common.h packed_index; 8 aligned columns stay contiguous)
      *(u16x8*)(y + (pack ? packed_index(row, ci * 8, ldy) : (int64_t)row * ldy + ci * 8)) = o;
    }
  }
}

void launch_rmsnorm(const u16* x, int64_t ldx, const int32_t* row_index, int row_sub, const u16* w,
                    u16* y, int64_t ldy, int M, int N, float eps, hipStream_t s, bool pack_out,
                    unsigned long long* zero_slots, int n_slots, const NormPrologue* pro_in) {
  if (!zero_slots || M > 64) n_slots = 0;
  const NormPrologue pro = pro_in ? *pro_in : NormPrologue{};
  const int pk = pack_out ? 1 : 0;
  int ch = (N / 8 + 255) / 256;
  dim3 g(M), b(256);
  if (ch <= 1)
    hipLaunchKernelGGL(rmsnorm_kernel<1>, g, b, 0, s, x, ldx, row_index, row_sub, w, y, ldy, N, eps, pk,
                       zero_slots, n_slots, pro);
  else if (ch <= 2)
    hipLaunchKernelGGL(rmsnorm_kernel<2>, g, b, 0, s, x, ldx, row_index, row_sub, w, y, ldy, N, eps, pk,
                       zero_slots, n_slots, pro);
  else if (ch <= 4)
    hipLaunchKernelGGL(rmsnorm_kernel<4>, g, b, 0, s, x, ldx, row_index, row_sub, w, y, ldy, N, eps, pk,
                       zero_slots, n_slots, pro);
  else
    hipLaunchKernelGGL(rmsnorm_kernel<8>, g, b, 0, s, x, ldx, row_index, row_sub, w, y, ldy, N, eps, pk,
                       zero_slots, n_slots, pro);
}

// ------------------------------------------------------------------ rope table
// cos/sin[pos][i] for i < 64, HF default rope: freq = pos * inv_freq[i] in fp32
// (client.py:56-71); stored as bf16 exactly like `cos.to(dtype=x.dtype)`.
__global__ void rope_table_kernel(const float* __restrict__ inv_freq, int max_pos,
                                  u16* __restrict__ cos_t, u16* __restrict__ sin_t) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)max_pos * 64) return;
  int pos = (int)(i >> 6), k = (int)(i & 63);
  float a = __fmul_rn((float)pos, inv_freq[k]);
  cos_t[i] = f2bf(cosf(a));
  sin_t[i] = f2bf(sinf(a));
}

void launch_rope_table(const float* inv_freq, int max_pos, u16* cos_t, u16* sin_t, hipStream_t s) {
  int64_t n = (int64_t)max_pos * 64;
  hipLaunchKernelGGL(rope_table_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                     inv_freq, max_pos, cos_t, sin_t);
}

// ------------------------------------------------------------------ QK-norm + RoPE + KV write
// qkv row layout: [q heads (H*128) | k heads (KV*128) | v heads (KV*128)].
// 16 threads per head, 8 dims per thread.  q -> q_out[M][H][128]; k, v -> paged cache.
__global__ __launch_bounds__(256) void qk_norm_rope_kv_kernel(
    const u16* __restrict__ qkv, int64_t ldqkv, const int32_t* __restrict__ positions,
    const int32_t* __restrict__ slots, const u16* __restrict__ qn_w, const u16* __restrict__ kn_w,
    const u16* __restrict__ cos_t, const u16* __restrict__ sin_t, u16* __restrict__ q_out,
    u16* __restrict__ kv_layer, int H, int KV, float eps) {
  int tok = blockIdx.y;
  int hh = blockIdx.x * 16 + (threadIdx.x >> 4);
  int c = threadIdx.x & 15;  // dims 8c .. 8c+7
  int nheads = H + 2 * KV;
  bool active = hh < nheads;
  int hsafe = active ? hh : 0;
  const u16* src = qkv + (int64_t)tok * ldqkv + (int64_t)hsafe * HEAD_DIM + c * 8;
  u16x8 raw = *(const u16x8*)src;
  float x[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = bf2f(raw[j]);
  int pos = positions[tok];
  int slot = slots ? slots[tok] : -1;

  if (hsafe < H + KV) {  // q or k head: RMSNorm over 128 dims, then RoPE (uniform per 16 lanes)
    const u16* nw = hsafe < H ? qn_w : kn_w;
    float ss = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) ss += x[j] * x[j];
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 16);
    float inv = 1.0f / sqrtf(ss / 128.0f + eps);
    u16x8 wv = *(const u16x8*)(nw + c * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = rbf(bf2f(wv[j]) * rbf(x[j] * inv));
    // rotate_half partner: dims d+64 (c < 8) or d-64 (c >= 8) live in lane c ^ 8
    float pr[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) pr[j] = __shfl_xor(x[j], 8, 16);
    int ci = (c & 7) * 8;
    u16x8 cv = *(const u16x8*)(cos_t + (int64_t)pos * 64 + ci);
    u16x8 sv = *(const u16x8*)(sin_t + (int64_t)pos * 64 + ci);
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float rot = c < 8 ? -pr[j] : pr[j];
      o[j] = f2bf(rbf(x[j] * bf2f(cv[j])) + rbf(rot * bf2f(sv[j])));
    }
    if (active) {
      if (hsafe < H) {
        *(u16x8*)(q_out + ((int64_t)tok * H + hsafe) * HEAD_DIM + c * 8) = o;
      } else if (slot >= 0) {
        int g = hsafe - H;
        int page = slot >> 6, s = slot & 63;
        u16* blk = kv_layer + kv_block(page, 0, g, KV);
        int tb = s >> 4, ks = c >> 2, lane = (s & 15) + 16 * (c & 3);
        *(u16x8*)(blk + ((tb * 4 + ks) * 64 + lane) * 8) = o;
      }
    }
  } else if (active && slot >= 0) {  // v head: scatter into the V^T tile layout
    int g = hsafe - H - KV;
    int page = slot >> 6, s = slot & 63;
    u16* blk = kv_layer + kv_block(page, 1, g, KV);
    int kt = s >> 5, tp = s & 31;
    int gg = tp < 16 ? (tp >> 2) : ((tp - 16) >> 2);
    int jj = tp < 16 ? (tp & 3) : 4 + ((tp - 16) & 3);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      int d = c * 8 + j;
      int db = d >> 4, lane = (d & 15) + 16 * gg;
      blk[((kt * 8 + db) * 64 + lane) * 8 + jj] = raw[j];
    }
  }
}

void launch_qk_norm_rope_kv(const u16* qkv, int64_t ldqkv, const int32_t* positions,
                            const int32_t* slots, const u16* qn_w, const u16* kn_w,
                            const u16* cos_t, const u16* sin_t, u16* q_out, u16* kv_layer, int M,
                            int H, int KV, float eps, hipStream_t s) {
  dim3 g((H + 2 * KV + 15) / 16, M);
  hipLaunchKernelGGL(qk_norm_rope_kv_kernel, g, dim3(256), 0, s, qkv, ldqkv, positions, slots,
                     qn_w, kn_w, cos_t, sin_t, q_out, kv_layer, H, KV, eps);
}

// ------------------------------------------------------------------ embedding gather
__global__ void embed_kernel(const int32_t* __restrict__ ids, const u16* __restrict__ table,
                             int N, int vocab, u16* __restrict__ out, int32_t* __restrict__ err) {
  int row = blockIdx.x;
  int id = ids[row];
  if (id < 0 || id >= vocab) {
    if (threadIdx.x == 0) atomicOr(err, 1);
    id = 0;
  }
  for (int c = threadIdx.x; c < N / 8; c += blockDim.x)
    *(u16x8*)(out + (int64_t)row * N + c * 8) = *(const u16x8*)(table + (int64_t)id * N + c * 8);
}

void launch_embed(const int32_t* ids, const u16* table, int M, int N, int vocab, u16* out,
                  int32_t* err, hipStream_t s) {
  hipLaunchKernelGGL(embed_kernel, dim3(M), dim3(256), 0, s, ids, table, N, vocab, out, err);
}

// ------------------------------------------------------------------ decode-step advance (own launch)
__global__ void decode_advance_kernel(int32_t* __restrict__ positions, int32_t* __restrict__ slots,
                                      int32_t* __restrict__ ctx_lens, const int32_t* __restrict__ block_table,
                                      int max_pages, int B, int32_t* __restrict__ err) {
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < B) decode_advance_one(positions, slots, ctx_lens, block_table, max_pages, b, err);
}

void launch_decode_advance(int32_t* positions, int32_t* slots, int32_t* ctx_lens, const int32_t* block_table,
                           int max_pages, int B, int32_t* err, hipStream_t s) {
  hipLaunchKernelGGL(decode_advance_kernel, dim3((B + 63) / 64), dim3(64), 0, s, positions, slots, ctx_lens,
                     block_table, max_pages, B, err);
}

// ------------------------------------------------------------------ argmax key decode
// key = (float_key(bf16 logit) << 32) | (0xFFFFFFFF - index): max key = max logit, lowest index
__global__ void argmax_decode_kernel(const unsigned long long* __restrict__ keys, int B,
                                     int32_t* __restrict__ ids) {
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < B) ids[b] = (int32_t)(0xFFFFFFFFu - (uint32_t)(keys[b] & 0xFFFFFFFFull));
}

void launch_argmax_decode(const unsigned long long* keys, int B, int32_t* ids, hipStream_t s) {
  hipLaunchKernelGGL(argmax_decode_kernel, dim3((B + 63) / 64), dim3(64), 0, s, keys, B, ids);
}

// ------------------------------------------------------------------ q/k/v slice reduction
// The bf16 q/k/v rows of a decode call from the split-K projection's fp32 slices
// (launch_gemm_decode_partial: [ksl][M][N]), summed exactly as the fused decode attention sums
// them (attention.hip qkv8: 0 + slice 0 + ... + slice 3, zeros past ksl, rounded once) -- the
// raw q/k/v part of a q/k/v|attention boundary's record.
__global__ __launch_bounds__(256) void qkv_reduce_kernel(const float* __restrict__ part, int ksl, int M, int N,
                                                         u16* __restrict__ out) {
  const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  const int64_t n = (int64_t)M * N;
  if (i >= n) return;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int sl = 0; sl < 4; ++sl) {
    const f32x4 p = sl < ksl ? *(const f32x4*)(part + (int64_t)sl * n + i) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] += p[j];
  }
  u16x4 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) o[j] = f2bf(acc[j]);
  *(u16x4*)(out + i) = o;
}

void launch_qkv_reduce(const float* part, int ksl, int M, int N, u16* out, hipStream_t s) {
  const int64_t n4 = ((int64_t)M * N + 3) / 4;
  hipLaunchKernelGGL(qkv_reduce_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, s, part, ksl, M, N, out);
}
