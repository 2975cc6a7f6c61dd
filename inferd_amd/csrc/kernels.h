// Host-side launchers of the span kernels (internal C++ interface; the public
// boundary is the extern "C" API in include/inferd_span.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

typedef unsigned short u16;

enum GemmEpilogue {
  EPI_NONE = 0,    // C = bf16(acc)
  EPI_RESID = 1,   // C = bf16(bf16(acc) + R)              (o_proj / down_proj + residual)
  EPI_SILU = 2,    // C = bf16(bf16(silu(bf16(g))) * bf16(u)) with [gate; up] packed weight
  EPI_ARGMAX = 3,  // per-row partial argmax keys of bf16(acc) (+ optional bf16 logits in C)
  EPI_PARTIAL = 4, // internal: fp32 K-slice partials (+ row sums of squares), reduced by the consumer
  EPI_QKV = 5,     // internal: prefill q/k/v projection with q/k RMSNorm + RoPE and the K/V cache write
};

// EPI_QKV epilogue operands (qk_norm_rope_kv_kernel's, applied to the GEMM's tile in registers)
struct QkvEpilogue {
  const int32_t* positions;
  const int32_t* slots;
  const u16* qn_w;
  const u16* kn_w;
  const u16* cos_t;
  const u16* sin_t;
  u16* q_out;
  u16* kv_layer;
  int H, KV;
  float eps;
};

// elementwise.hip
void launch_weightgen(u16* dst, int64_t n, uint64_t key, float scale, float center, hipStream_t s);
void launch_pack(const u16* src, int64_t ld, int N, int K, u16* dst, hipStream_t s);
void launch_unpack(const u16* src, int N, int K, u16* dst, hipStream_t s);
// Work a decode step's first RMSNorm launch can take over from two launches of its own (each
// a ~4.5 us node of the decode graph): the embedding gather (ids != null: row r of x is
// table[ids[r]], also written to x_out, ldx = N; bad ids set err bit 0 like embed_kernel) and
// the graph's scheduler step (positions != null: decode_advance_kernel's update by workgroup
// 0 -- nothing in the norm reads them).
struct NormPrologue {
  const int32_t* ids = nullptr;
  const u16* table = nullptr;
  int vocab = 0;
  int32_t* err = nullptr;
  u16* x_out = nullptr;
  int32_t* positions = nullptr;
  int32_t* slots = nullptr;
  int32_t* ctx_lens = nullptr;
  const int32_t* block_table = nullptr;
  int max_pages = 0, B = 0;
};
// the same prologue work (scheduler step, SSQ slot zeroing for rows < M <= 64) as a launch of its
// own, for a span whose first launch is not an RMSNorm
// bf16 q/k/v rows from decode split-K slices ([ksl][M][N] fp32, M * N % 4 == 0), summed in the
// fused decode attention's order
void launch_qkv_reduce(const float* part, int ksl, int M, int N, u16* out, hipStream_t s);
void launch_step_prologue(unsigned long long* zero_slots, int n_slots, int M, const NormPrologue* pro,
                          hipStream_t s);
// zero_slots: rows < M of n_slots SSQ slots (kernels.h DecodeNorm) are zeroed too, or null
void launch_rmsnorm(const u16* x, int64_t ldx, const int32_t* row_index, int row_sub, const u16* w,
                    u16* y, int64_t ldy, int M, int N, float eps, hipStream_t s, bool pack_out = false,
                    unsigned long long* zero_slots = nullptr, int n_slots = 0, const NormPrologue* pro = nullptr);
void launch_rope_table(const float* inv_freq, int max_pos, u16* cos_t, u16* sin_t, hipStream_t s);
void launch_qk_norm_rope_kv(const u16* qkv, int64_t ldqkv, const int32_t* positions,
                            const int32_t* slots, const u16* qn_w, const u16* kn_w,
                            const u16* cos_t, const u16* sin_t, u16* q_out, u16* kv_layer, int M,
                            int H, int KV, float eps, hipStream_t s);
void launch_embed(const int32_t* ids, const u16* table, int M, int N, int vocab, u16* out,
                  int32_t* err, hipStream_t s);
void launch_argmax_decode(const unsigned long long* keys, int B, int32_t* ids, hipStream_t s);
void launch_decode_advance(int32_t* positions, int32_t* slots, int32_t* ctx_lens, const int32_t* block_table,
                           int max_pages, int B, int32_t* err, hipStream_t s);

// gemm.hip.  Wp is fragment-packed (common.h).  N counts OUTPUT columns: for EPI_SILU the
// packed weight holds 2N rows ([gate; up]).  For EPI_ARGMAX `partial` receives
// (N/16) x M keys and `amax_keys` the per-row reduction (M <= 64).
bool gemm_uses_tiled(int M, int N, int K, int epi);
// RMSNorm modes of the decode (M <= 64) GEMV
enum { DN_NONE = 0, DN_EXACT = 2 };
// DN_EXACT: Qwen3RMSNorm at the reference's rounding points applied to A inside the GEMV,
// A' = bf16(w * bf16(A * r)), r = 1 / sqrt(ssq[row] / K + eps).  ssq[row] comes from the kernel
// that produced A (launch_gemm's ssq_out on an EPI_RESID GEMV) as an exact fixed-point sum in one
// SSQ slot: each producer workgroup adds its 16-column tile's fp32 row sums of squares, split into
// hi = floor(q * 2^8) and lo = frac(q * 2^8) * 2^32, to shard (tile % SSQ_SHARDS) with no-return
// 64-bit atomics; integer adds commute, so the sum is order-independent (deterministic) and exact
// to 2^-40.  Slot layout: [SSQ_SHARDS][hi | lo][64 rows] u64; a slot must be zero before its
// producer runs (launch_rmsnorm's `zero_slots`).
#define SSQ_SHARDS 8
#define SSQ_SLOT_WORDS (SSQ_SHARDS * 64 * 2)
struct DecodeNorm {
  int mode;
  float eps;
  const unsigned long long* ssq;  // the slot the producer of A filled
  const u16* w;
};
// Per-span GEMM workspace: the prefill tail split's fp32 partials and tickets, allocated once
// at span creation (gemm_ws_alloc: the split's fixed maximum, 8 XCDs x 32 slices of a 256x256
// fp32 tile = 64 MiB, and 512 zeroed tickets), so a forward call never allocates and a graph
// capture may contain the split (one workspace per span: spans on different streams never
// share tickets).  split = 0 disables the tail split (spans whose max_tokens < 512 never split).
struct GemmWs {
  float* ws = nullptr;
  unsigned* cnt = nullptr;
  int split = 1;
};
int gemm_ws_alloc(GemmWs* w);  // hipError_t as int
void gemm_ws_free(GemmWs* w);
// ssq_out (EPI_RESID, M <= 64): the SSQ slot (above) that receives the row sums of squares of
// the stored outputs -- the DecodeNorm input of the next normed GEMV.  Returns false, launching
// nothing, for a combination no body implements (DN_EXACT or ssq_out with M > 64, DN_EXACT with
// EPI_RESID): the caller must fail rather than let a consumer read an unfilled SSQ slot.
// up_tiles (decode EPI_SILU only, else refused): the [gate; up] weight is a column range of a
// wider projection -- Wp points at its first gate tile and its up tiles sit up_tiles 16-column
// tiles after the gate tiles (the whole projection's gate width); 0 = N / 16
bool launch_gemm(const u16* A, int64_t lda, const u16* Wp, int M, int N, int K, u16* C, int64_t ldc,
                 const u16* R, int64_t ldr, int epi, unsigned long long* keys, hipStream_t s,
                 const GemmWs* ws = nullptr, const DecodeNorm* dn = nullptr, unsigned long long* ssq_out = nullptr,
                 int pack = 0, int up_tiles = 0);
// launch_gemm `pack` bits (decode path, M <= 64 only; common.h packed_index): A is read
// fragment-packed / the EPI_SILU or EPI_RESID output C is written so / the EPI_RESID residual
// R is read so
enum { GEMM_PACK_A = 1, GEMM_PACK_C = 2, GEMM_PACK_R = 4 };
// prefill q/k/v projection fused with q/k RMSNorm + RoPE and the K/V cache write (the
// persistent GEMM's epilogue); returns false, launching nothing, where that body does not
// apply (the caller then runs launch_gemm + launch_qk_norm_rope_kv)
bool launch_gemm_qkv_fused(const u16* A, int64_t lda, const u16* Wp, int M, int N, int K, const QkvEpilogue& e,
                           hipStream_t s);
// decode q/k/v with K split over `kslices` (M <= 16): part [kslices][M][N] fp32; the fused
// decode attention reduces them
void launch_gemm_decode_partial(const u16* A, int64_t lda, const u16* Wp, int M, int N, int K, int kslices,
                                float* part, const DecodeNorm& norm, hipStream_t s, int pack = 0);
void launch_argmax_reduce(const unsigned long long* partial, int n_tiles, int M,
                          int32_t* ids, hipStream_t s);
// vocab-parallel lm_head: a shard's per-row max key with its first vocabulary row folded into the
// index part, and the combine over shards (inferd_span_head_shard / inferd_argmax_combine)
void launch_argmax_keys(const unsigned long long* partial, int n_tiles, int M, int col0,
                        const unsigned long long* keys_in, unsigned long long* keys_out, int32_t* ids, hipStream_t s);
void launch_argmax_combine(const unsigned long long* keys, int n_parts, int rows, int32_t* ids, hipStream_t s);

// attention.hip
struct AttnBatch {
  const int32_t* seq_start;    // [B+1] first token row of each sequence
  const int32_t* positions;    // [M]
  const int32_t* ctx_lens;     // [B] keys visible to the LAST token of the sequence
  const int32_t* block_table;  // [B][max_pages]
  int max_pages;
  int B;
  int M;
  int max_q_len;
  int max_ctx;
};
// q [M][H][128] bf16 -> out [M][H*128] bf16.  kv_layer: this layer's pool base.
void launch_attn_decode(const u16* q, const u16* kv_layer, const AttnBatch& b, int H, int KV,
                        float scale, u16* out, float* ws, hipStream_t s);
// Decode attention with the token's QK-norm + RoPE + K/V cache write fused in (replaces
// launch_qk_norm_rope_kv + launch_attn_decode on the decode path): qkv is the raw
// [M][(H+2KV)*128] projection output.
// With `part` non-null the q/k/v come from launch_gemm_decode_partial's fp32 K-slices
// (part [ksl][M][ldqkv], already normed) instead of the bf16 rows `qkv`.
// pack_out: `out` is written fragment-packed (common.h packed_index, whole 16-row tiles).
void launch_attn_decode_fused(const u16* qkv, int64_t ldqkv, const u16* qn_w, const u16* kn_w, const u16* cos_t,
                              const u16* sin_t, float eps, u16* kv_layer, const AttnBatch& b, int H, int KV,
                              float scale, u16* out, float* ws, hipStream_t s, const float* part = nullptr,
                              int ksl = 0, bool pack_out = false);
size_t attn_decode_ws_bytes(int B, int H, int max_ctx);
void launch_attn_prefill(const u16* q, const u16* kv_layer, const AttnBatch& b, int H, int KV,
                         float scale, u16* out, hipStream_t s);

// sets the thread-local message of inferd_last_error() and returns `code` (span.hip)
int inferd_fail(int code, const std::string& msg);
