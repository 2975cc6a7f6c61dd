/*
 * inferd_span.h -- C-ABI of the MI355X (gfx950) Qwen3 layer-span engine.
 *
 * This is the drop-in boundary underneath InferD's span API.  The reference has no
 * native code: its span compute is PyTorch/transformers called from Python
 * (petals/partitioned_models.py, models/qwen3/server/qwen3_server_module.py).  Each
 * entry point below names the reference interface it replaces.  The Python host side
 * (inferd_amd/partitioned_models.py, inferd_amd/qwen3_server.py) binds this header
 * with ctypes; INTEGRATION.md shows the binding.
 *
 * Conventions
 *  - Plain pointers and sizes only.  "device" pointers are HIP device memory; bf16
 *    tensors are raw 16-bit patterns, row-major, contiguous.
 *  - `stream` is a hipStream_t passed as void* (NULL = default stream).  Every call is
 *    stream-ordered and asynchronous; nothing here synchronises the device.
 *  - Every int-returning call returns INFERD_OK (0) or an INFERD_ERR_* code and leaves
 *    a thread-local message readable through inferd_last_error().  No exception
 *    crosses the ABI (the Python wrapper raises RuntimeError, as an exception in
 *    PartitionedQwen2.forward propagates through task.py:54 to aiohttp as HTTP 500).
 *  - Threading: one span handle is used from one host thread at a time (the reference
 *    runs forward synchronously on the asyncio loop thread, task_scheduler.py:18).
 */
#ifndef INFERD_SPAN_H
#define INFERD_SPAN_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define INFERD_OK 0
#define INFERD_ERR_ARG 1   /* bad argument / shape / unsupported configuration */
#define INFERD_ERR_HIP 2   /* HIP runtime error (allocation, launch) */
#define INFERD_ERR_STATE 3 /* handle not initialised / weights not ready (see set_weight) */
#define INFERD_ERR_NOMEM 4 /* KV page pool exhausted (inferd_kv_reserve; nothing was taken) */

#define INFERD_KV_PAGE_TOKENS 64

/* GEMM epilogues (inferd_gemm) */
#define INFERD_EPI_NONE 0  /* C = bf16(A W^T)                                      */
#define INFERD_EPI_RESID 1 /* C = bf16(bf16(A W^T) + R)                            */
#define INFERD_EPI_SILU 2  /* W = [gate; up] (2N x K): C = bf16(silu(g) * u)       */

/* Model + span geometry.  Replaces the span construction of split_model.py:92-108
 * (span = layers[start_layer .. end_layer] of petals/inferd.yaml, plus embed for the
 * first stage and final norm + lm_head for the last) and Qwen3Server(start, end)
 * (qwen3_server_module.py:209-224).  Model constants: qwen3_config.py:10-24. */
typedef struct InferdSpanConfig {
  int32_t hidden;         /* HIDDEN_SIZE */
  int32_t intermediate;   /* INTERMEDIATE_SIZE */
  int32_t heads;          /* NUM_ATTENTION_HEADS */
  int32_t kv_heads;       /* NUM_KEY_VALUE_HEADS */
  int32_t head_dim;       /* HEAD_DIM (must be 128) */
  int32_t vocab;          /* VOCAB_SIZE */
  int32_t first_layer;    /* global index of the span's first layer (start_layer) */
  int32_t n_layers;       /* end_layer - start_layer + 1 */
  int32_t has_embed;      /* FirstStage: owns embed_tokens */
  int32_t has_lm_head;    /* LastStage: owns final norm + lm_head */
  float rms_eps;          /* RMS_NORM_EPS */
  float rope_theta;       /* ROPE_THETA */
  int32_t max_positions;  /* MAX_POSITION_EMBEDDINGS (rope table rows) */
  int32_t kv_pages;       /* KV pool capacity, in INFERD_KV_PAGE_TOKENS-token pages */
  int32_t max_tokens;     /* activation workspace rows (tokens per forward call) */
  int32_t max_seqs;       /* sequences per forward call */
  /* Sub-layer stage boundaries (ABI 3; q/k/v boundaries ABI 4).  The reference cuts spans at layer boundaries only
   * (split_model.py:92-108); a pipeline balanced to the last stage's lm_head needs a finer
   * cut.  A decoder layer (qwen3_server_module.py:179-206) is two halves: attention
   * (input_layernorm .. o_proj + residual) and MLP (post_attention_layernorm .. down_proj +
   * residual).  The hidden state handed over between the halves is the residual stream h1,
   * the same bf16 [n_tokens][hidden] tensor a layer boundary hands over. */
  int32_t skip_first_attn; /* the span begins at its first layer's MLP half (input: h1; no embed) */
  int32_t skip_last_mlp;   /* the span ends after its last layer's attention half (output: h1; no lm_head) */
  /* A finer boundary inside the gate/up projection, for calls of <= 64 rows (any kind, decode or
   * a short prefill): the span before the boundary also computes gate/up columns [0, c) of that
   * layer's SwiGLU product `act`, the span after it the columns [c, intermediate) and the down
   * projection.  Every call of <= 64 rows then hands over a RECORD: h1 bf16 [n_tokens][hidden]
   * row-major, followed by act bf16 [ceil(n_tokens/16)*16][intermediate] fragment-packed (columns
   * [0, c) filled).  The receiving span completes the other columns IN PLACE in x_in's record (x_in
   * is written although the API passes it as const void*), so both sides must size x_in / x_out
   * for the whole record (the C-ABI does not check buffer sizes; the torch extension does).
   * Calls of more than 64 rows hand over h1 only and the receiving span computes the whole MLP.
   * Values and rounding points are those of one span: act columns are independent, down runs
   * whole on one side.  c: 0 = none, else a multiple of 128 below intermediate. */
  int32_t gateup_split_first; /* with skip_first_attn: columns [0, c) arrive in x_in's record (written in place) */
  int32_t gateup_split_last;  /* with skip_last_mlp: columns [0, c) are computed into x_out's record */
  /* A boundary between a layer's attention kernel and its o projection: the span before it
   * runs input_layernorm, q/k/v and the attention of that layer (its K/V pages live there),
   * the span after it starts with o_proj + residual.  The hand-off is a RECORD: the layer's
   * input residual x bf16 [n_tokens][hidden] row-major, followed by the attention output bf16
   * [rows][heads * 128] -- fragment-packed over ceil(n_tokens/16)*16 rows in a pure decode call
   * (every sequence one new token), row-major over n_tokens rows otherwise.  0 or 1. */
  int32_t o_split_first; /* the span starts at its first layer's o projection (x_in: the record) */
  int32_t o_split_last;  /* the span ends before its last layer's o projection (x_out: the record) */
  /* A boundary between a layer's q/k/v projection and its attention kernel (ABI 4): the span
   * before it runs that layer's input_layernorm and q/k/v projection, the span after it the
   * attention (its K/V pages live there), o_proj and the MLP.  In a pure decode call the
   * hand-off is a RECORD: the layer's input residual x bf16 [n_tokens][hidden] row-major,
   * followed by the raw q/k/v projection output bf16 [n_tokens][(heads + 2 kv_heads) * 128]
   * row-major (before QK-norm and RoPE: the receiver's attention applies them and writes the
   * cache).  Other calls hand over x only and the receiving span runs the whole layer (it owns
   * the layer's input_layernorm and q/k/v weights too).  0 or 1. */
  int32_t qkv_split_first; /* the span starts at its first layer's attention (x_in: the record) */
  int32_t qkv_split_last;  /* the span ends after its last layer's q/k/v projection (x_out: the record) */
  /* Vocab-parallel lm_head (ABI 5).  The reference's last span owns the whole lm_head
   * (split_model.py:97-102) and takes argmax(logits[:, -1]) (partitioned_models.py:95-96,162).
   * In a pipeline that 1.24 GB GEMV sits on one stage; these fields spread it over the stages:
   * the model's last span keeps only the final norm (final_norm_out) and hands out the normed
   * last rows, every span may own a contiguous shard of lm_head rows, inferd_span_head_shard
   * reduces a shard to one (max logit, first index) key per row, and inferd_argmax_combine
   * takes the max over the shards' keys -- torch.argmax's value and lowest-index tie-break, bit
   * for bit (a logit's value does not depend on which shard computes it: one 16-column GEMV tile
   * per workgroup over the whole K range, tiles aligned to 16 rows). */
  int32_t head_first;     /* first lm_head row of this span's shard (a multiple of 16) */
  int32_t head_rows;      /* rows of the shard (a multiple of 16; 0 = none).  Not with has_lm_head,
                             which owns all rows (and may also be reduced by inferd_span_head_shard) */
  int32_t final_norm_out; /* the model's last span, head vocab-parallel: owns the final norm (weight
                             "norm"; no lm_head); a forward with x_out writes the final-normed last
                             row of each sequence there, fragment-packed over ceil(n_seqs/16)*16 rows
                             ([n_seqs <= 64][hidden]: the A operand of inferd_span_head_shard), instead
                             of the last layer's hidden rows.  Ends at a layer boundary. */
} InferdSpanConfig;

/* One forward call's batch: n_seqs sequences, their new tokens concatenated
 * (n_tokens rows).  All arrays are device int32.  The KV cache of every sequence is a
 * list of pages (block_table row); a token at `positions[i]` writes its K/V to global
 * slot `slots[i]` = page * 64 + offset and attends to keys 0..positions[i] of its
 * sequence.  This single descriptor covers the petals full-recompute call
 * (partitioned_models.py:139-143: positions 0..T-1, fresh pages) and the cached
 * prefill / single-token decode of Qwen3Server.send (qwen3_server_module.py:237-255,
 * client.py:244-266). */
typedef struct InferdBatch {
  int32_t n_seqs;
  int32_t n_tokens;
  int32_t max_q_len;           /* max new tokens of one sequence */
  int32_t max_ctx_len;         /* max of ctx_lens */
  int32_t max_pages;           /* block_table row stride */
  int32_t decode;              /* 1 iff every sequence has exactly one new token */
  const int32_t* seq_start;    /* [n_seqs + 1] token-row offsets */
  const int32_t* positions;    /* [n_tokens] */
  const int32_t* slots;        /* [n_tokens] */
  const int32_t* ctx_lens;     /* [n_seqs]: positions[last token] + 1 */
  const int32_t* block_table;  /* [n_seqs][max_pages] */
} InferdBatch;

typedef struct InferdSpan InferdSpan;

const char* inferd_last_error(void);
int inferd_abi_version(void);

/* ---- span lifetime (replaces torch.load of the pickled stage module,
 *      partitioned_models.py:112-117, and Qwen3Server.__init__/_load_weights,
 *      qwen3_server_module.py:209-235) ---------------------------------------------- */
int inferd_span_create(const InferdSpanConfig* cfg, InferdSpan** out);
void inferd_span_destroy(InferdSpan* span);
/* the configuration the span was created with (hosts size their buffers from it) */
int inferd_span_get_config(const InferdSpan* span, InferdSpanConfig* out);
/* bf16 elements the x_in (which = 0) / x_out (which = 1) buffer of a forward or step call of
 * n_tokens rows over n_seqs sequences (decode: a pure decode call) must hold: the hidden rows plus
 * the record a sub-layer boundary hands over, or a final_norm_out span's normed rows.  A pure
 * function of the config (no span needed); -1 on bad arguments.  inferd_span_forward and
 * inferd_span_step take plain pointers and cannot check sizes: size the buffers with this. */
int64_t inferd_span_io_elems(const InferdSpanConfig* cfg, int32_t n_tokens, int32_t n_seqs, int32_t decode,
                             int32_t which);

/* Fill every weight of the span from the counter-based generator (oracle/weightgen.py
 * defines the same values) -- the offline stand-in for the HF checkpoint. */
int inferd_span_init_synthetic(InferdSpan* span, uint64_t seed, void* stream);

/* Load one weight from a row-major device bf16 tensor.  `layer` is span-local
 * (0..n_layers-1) or -1 for embed_tokens / norm / lm_head.  `name` uses the reference's
 * state-dict leaf names (qwen3_server_module.py:101-124, :169-176):
 * q_proj k_proj v_proj o_proj q_norm k_norm input_layernorm post_attention_layernorm
 * gate_proj up_proj down_proj | embed_tokens norm lm_head.  Projections are packed into
 * the device fragment layout (fused [q;k;v] and [gate;up]).  The RMSNorms run at the
 * reference's rounding points (bf16(w * bf16(x * rsqrt(mean(x^2) + eps)))) from the norm
 * weights as set, so weights may be set in any order. */
int inferd_span_set_weight(InferdSpan* span, int32_t layer, const char* name,
                           const void* src, int64_t rows, int64_t cols, void* stream);

/* Span forward.  Replaces FirstStage/StageInner/LastStage.forward
 * (partitioned_models.py:47-57, :66-75, :86-97) and Qwen3Server.send
 * (qwen3_server_module.py:237-255).
 *   ids       first span only: device int32 [n_tokens] token ids (embed gather)
 *   x_in      other spans: device bf16 [n_tokens][hidden] hidden states
 *   x_out     optional device bf16 [n_tokens][hidden]: hidden after the last layer
 *   next_ids  last span only, optional: device int32 [n_seqs] greedy token of each
 *             sequence's last row (norm -> lm_head -> argmax, partitioned_models.py:162);
 *             ties resolve to the lowest index like torch.argmax
 *   logits    last span only, optional: device bf16 [n_seqs][vocab] last-row logits
 *   layer_out optional device bf16 [n_layers][n_tokens][hidden] per-layer capture */
int inferd_span_forward(InferdSpan* span, const InferdBatch* batch, const int32_t* ids,
                        const void* x_in, void* x_out, int32_t* next_ids, void* logits,
                        void* layer_out, void* stream);

/* Final norm + lm_head over `rows` rows of bf16 hidden states x -> bf16 logits [rows][vocab]
 * (LastStage.forward returns logits for all T positions, partitioned_models.py:95-96;
 * inferd_span_forward computes the last row of each sequence only).  Last span only,
 * rows <= max_tokens. */
int inferd_span_lm_head(InferdSpan* span, const void* x, int32_t rows, void* logits, void* stream);

/* Vocab-parallel greedy head (ABI 5; InferdSpanConfig head_first / head_rows): the span's lm_head
 * shard over `rows` (<= 64) final-normed rows `normed` (bf16, fragment-packed over
 * ceil(rows/16)*16 rows: what a final_norm_out span's forward writes to x_out).  A row's KEY is
 * (order(bf16 logit) << 32 | (0xFFFFFFFF - c)) maximised over columns c, c the GLOBAL vocabulary
 * index: the max key is the max logit, ties to the lowest index (torch.argmax).  All outputs are
 * optional and device-side:
 *   keys_in   uint64 [rows]: the running max key of the shards before this one (NULL: none)
 *   keys_out  uint64 [rows]: max(keys_in, this shard's key) (may alias keys_in)
 *   ids       int32 [rows]: the greedy token of that max key
 *   logits    bf16 [rows][head_rows] row-major: the shard's columns
 * Chaining the call over the shards in any order (keys_out -> the next keys_in) and taking ids at
 * the end gives argmax(norm(x) @ lm_head^T) of the whole vocabulary.  A span with has_lm_head
 * reduces all rows.  Replaces, split over the stages, LastStage's lm_head + argmax
 * (partitioned_models.py:95-96,162). */
int inferd_span_head_shard(InferdSpan* span, const void* normed, int32_t rows, const uint64_t* keys_in,
                           uint64_t* keys_out, int32_t* ids, void* logits, void* stream);
/* ids[r] = the index in the max key over n_parts shards' keys [n_parts][rows] (device uint64):
 * the greedy token, ties to the lowest index as torch.argmax.  Device int32 ids [rows]. */
int inferd_argmax_combine(const uint64_t* keys, int32_t n_parts, int32_t rows, int32_t* ids, void* stream);

/* Decode graphs.  Captures one span forward of `batch` (same arguments as
 * inferd_span_forward; `logits`, last span only, optional: bf16 [n_seqs][vocab] last-row
 * logits of every replay) into a HIP graph.  With advance = 1 the graph starts with a
 * device-side scheduler step: for every sequence b the new token goes to position
 * ctx_lens[b], its slot comes from the block table, and ctx_lens[b] grows by one -- the
 * batch arrays are mutated in place, so repeated launches walk the sequences forward one
 * token per launch with no host work (build the batch with inferd_kv_build_decode_batch, which
 * reserves the pages and sets ctx_lens / max_ctx_len as this step expects; sequences running out
 * of pages set error flag bit 1).
 * `ids` and `next_ids` may be the same buffer (the step reads ids first).  Replaces the
 * per-token client loop over the chain (client.py:244-266, send_message.py:46-60). */
typedef struct InferdGraph InferdGraph;
int inferd_span_graph_capture(InferdSpan* span, const InferdBatch* batch, int32_t advance,
                              const int32_t* ids, const void* x_in, void* x_out, int32_t* next_ids,
                              void* logits, void* stream, InferdGraph** out);
int inferd_graph_launch(InferdGraph* graph, void* stream);
void inferd_graph_destroy(InferdGraph* graph);
/* The work of one replay of such a graph, launched eagerly on `stream`: the device-side
 * scheduler step (advance = 1, the same in-place batch update) and the span forward, kernel by
 * kernel, with the replay's arguments.  Measured against graph replays of a 5-layer Qwen3-8B
 * stage (profiles/r05/graph_gap_probe.json): 3-5 us less per step on the GPU, ~26 host kernel
 * launches instead of one graph launch. */
int inferd_span_step(InferdSpan* span, const InferdBatch* batch, int32_t advance, const int32_t* ids,
                     const void* x_in, void* x_out, int32_t* next_ids, void* logits, void* stream);
/* Sticky device error flags, read and cleared (synchronises the device).  Bit 0: a token id
 * outside [0, vocab) reached the embedding gather (it reads row 0 instead; the reference's
 * nn.Embedding raises IndexError, so the Python host validates ids before the launch);
 * bit 1: a decode graph ran past the pages reserved for it. */
int inferd_span_error_flags(InferdSpan* span, int32_t* flags);

/* Per-kernel-class timing: HIP events recorded on the launch stream around every kernel of
 * the forward (classes below), up to max_pairs pairs; stop() synchronises on the events
 * and returns the summed milliseconds and launch counts per class. */
#define INFERD_PROF_NORM 0
#define INFERD_PROF_QKV 1
#define INFERD_PROF_ROPE 2
#define INFERD_PROF_ATTN 3
#define INFERD_PROF_O 4
#define INFERD_PROF_GATEUP 5
#define INFERD_PROF_DOWN 6
#define INFERD_PROF_LMHEAD 7
#define INFERD_PROF_NCLASSES 8
int inferd_span_profile_start(InferdSpan* span, int32_t max_pairs);
int inferd_span_profile_stop(InferdSpan* span, double* total_ms, int32_t* counts, int32_t n_classes);

/* ---- KV page table (host-side, no device calls).  The per-sequence page lists and cached
 * lengths the span's paged KV pool is addressed by, and the InferdBatch a forward call reads.
 * Replaces the reference's per-session cache bookkeeping -- session_caches[session_id], a
 * DynamicCache appended to by every send (qwen3_server_module.py:220,253) -- and its position
 * arithmetic: positions 0..T-1 of a stateless recompute (partitioned_models.py:139-143),
 * cache_position = past .. past+T-1 of a cached step (client.py:244-266).  A sequence is any
 * caller-chosen 64-bit key; pages come lowest id first, so a fixed call sequence yields fixed
 * slots.  One table per span (kv_pages of its InferdSpanConfig). ------------------------ */
typedef struct InferdKvTable InferdKvTable;
int inferd_kv_create(int32_t n_pages, InferdKvTable** out);
void inferd_kv_destroy(InferdKvTable* table);
/* pages for n_new more tokens of `seq` (created empty if absent); all or nothing */
int inferd_kv_reserve(InferdKvTable* table, uint64_t seq, int32_t n_new);
/* n tokens of `seq` are now in the cache (within its reserved pages) */
int inferd_kv_advance(InferdKvTable* table, uint64_t seq, int32_t n);
/* the same for n_seqs sequences at once (a decode graph replay advances every sequence of its
 * batch by one token: one call per replay instead of one per sequence); all or nothing */
int inferd_kv_advance_many(InferdKvTable* table, const uint64_t* seqs, int32_t n_seqs, int32_t n);
/* drop `seq` and return its pages (absent: no-op) */
int inferd_kv_release(InferdKvTable* table, uint64_t seq);
/* cached length (-1: absent) and reserved page count of `seq` */
int inferd_kv_query(const InferdKvTable* table, uint64_t seq, int32_t* length, int32_t* n_pages);
int inferd_kv_pages(const InferdKvTable* table, uint64_t seq, int32_t* pages, int32_t cap);
int inferd_kv_free_pages(const InferdKvTable* table, int32_t* n_free);
/* The batch of n sequences, n_new[i] new tokens each (every seq reserved, each at most once):
 * batch_words() is the int32 count of its descriptor (-1 on a bad request); build_batch()
 * writes the words [seq_start | positions | slots | ctx_lens | block_table] to `host` and fills
 * `out` with pointers into `device_base`, where the caller copies the words before the
 * forward call.  Neither advances the sequences (inferd_kv_advance after the call). */
int64_t inferd_kv_batch_words(const InferdKvTable* table, const uint64_t* seqs, const int32_t* n_new,
                              int32_t n);
int inferd_kv_build_batch(const InferdKvTable* table, const uint64_t* seqs, const int32_t* n_new,
                          int32_t n, int32_t* host, int64_t words, const void* device_base,
                          InferdBatch* out);
/* The descriptor a decode graph (inferd_span_graph_capture, advance = 1) is captured on: pages
 * for n_steps more tokens of every sequence are reserved (all or nothing), positions and slots
 * start at 0 (the graph's scheduler step writes them), ctx_lens = the cached lengths and
 * max_ctx_len = the capacity (max length + n_steps).  decode_batch_words() is its int32 count
 * (-1 on a bad request).  The caller advances the table by one token per replay
 * (inferd_kv_advance_many), as the device does. */
int64_t inferd_kv_decode_batch_words(const InferdKvTable* table, const uint64_t* seqs, int32_t n,
                                     int32_t n_steps);
int inferd_kv_build_decode_batch(InferdKvTable* table, const uint64_t* seqs, int32_t n, int32_t n_steps,
                                 int32_t* host, int64_t words, const void* device_base, InferdBatch* out);

/* Device base pointer of one layer's KV pool: bf16
 * [pages / 16][kv_heads][pages % 16][K|V][64*128] (super-pages of 16 pages; a pool spans
 * whole super-pages, so callers of the single-op entry points below round their pool up to a
 * multiple of 16 pages).  `layer` is span-local; a layer the span runs only the MLP half of
 * (skip_first_attn) has no KV here (INFERD_ERR_ARG). */
int inferd_span_kv_layer(InferdSpan* span, int32_t layer, void** out);
/* Zero the KV pool. */
int inferd_span_kv_clear(InferdSpan* span, void* stream);

/* ---- single ops (the kernels the span forward chains; exported for parity tests) ---- */
/* splitmix64 counter generator: dst[i] = bf16(fl(fl(t_i * scale) + center)) */
int inferd_weightgen(void* dst, int64_t n, uint64_t seed, uint32_t tensor_id, float scale,
                     float center, void* stream);
/* row-major W[rows][cols] -> fragment-packed (rows % 16 == 0, cols % 32 == 0) and back */
int inferd_pack_weight(const void* src, int64_t rows, int64_t cols, void* dst, void* stream);
int inferd_unpack_weight(const void* src, int64_t rows, int64_t cols, void* dst, void* stream);
/* Qwen3RMSNorm.forward (qwen3_server_module.py:19-25) over rows of length cols */
int inferd_rmsnorm(const void* x, const void* w, void* y, int32_t rows, int32_t cols, float eps,
                   void* stream);
/* nn.Linear(bias=False) on a packed weight: C[m][n] = A[m][k] W[n][k]^T (+ epilogue) */
int inferd_gemm(const void* a, const void* w_packed, void* c, const void* resid, int32_t m,
                int32_t n, int32_t k, int32_t epilogue, void* stream);
/* rope cos/sin tables [max_pos][64] bf16 (HF default rope, client.py:56-71) */
int inferd_rope_table(float theta, int32_t head_dim, int32_t max_pos, void* cos_t, void* sin_t,
                      void* stream);
/* q/k RMSNorm + RoPE (qwen3_server_module.py:134-142) on a fused qkv row
 * [q (H*128) | k (KV*128) | v (KV*128)], q -> q_out [M][H][128], k/v -> paged cache
 * slots (DynamicCache.update, :144-148). slots may be NULL (no cache write). */
int inferd_qk_norm_rope_kv(const void* qkv, const int32_t* positions, const int32_t* slots,
                           const void* q_norm_w, const void* k_norm_w, const void* cos_t,
                           const void* sin_t, void* q_out, void* kv_layer, int32_t m,
                           int32_t heads, int32_t kv_heads, float eps, void* stream);
/* causal GQA attention of q [M][H][128] over the paged cache -> out [M][H*128].
 * Decode batches use `workspace` (inferd_attention_workspace_bytes); it must be
 * zero-filled before its first use, and every call leaves its counter block zero. */
int inferd_attention(const void* q, const void* kv_layer, const InferdBatch* batch,
                     int32_t heads, int32_t kv_heads, void* out, void* workspace,
                     int64_t workspace_bytes, void* stream);
int64_t inferd_attention_workspace_bytes(int32_t n_seqs, int32_t heads, int32_t max_ctx);

/* ---- Measurement probes (not on the span path; no reference counterpart).  SURVEY.md §8(d)
 * asks for the roofline peaks to be re-measured on the box beside the spec figures; bench.py
 * times these two launches with events on `stream` and reports both. */
/* streaming read of `bytes` at `buf`: n_wg workgroups of 512 lanes, each a contiguous run of
 * floor(bytes / 1024 / n_wg) KiB (pick bytes a multiple of 1024 * n_wg); `sink` (>= 2 KiB,
 * device) receives nothing for any realistic fill */
int inferd_probe_hbm_read(const void* buf, int64_t bytes, void* sink, int32_t n_wg, void* stream);
/* n_wg workgroups of 4 waves, each wave `iters` x 8 independent v_mfma_f32_16x16x32_bf16;
 * *flops = the launch's dense flop count (2*16*16*32 per MFMA) */
int inferd_probe_mfma(int32_t iters, int32_t n_wg, void* sink, void* stream, double* flops);

#ifdef __cplusplus
}
#endif
#endif /* INFERD_SPAN_H */
