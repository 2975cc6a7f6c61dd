// Span runtime + C-ABI (include/inferd_span.h).
//
// An InferdSpan owns everything one pipeline stage needs on its GPU: the layer weights
// in the fragment-packed layout (fused [q;k;v] and [gate;up]), the embedding table
// (first span), final norm + packed lm_head (last span), the bf16 rope tables, the
// paged KV pool and the activation workspace.  inferd_span_forward chains the kernels
// of one Qwen3 decoder layer per span layer
// (qwen3_server_module.py:179-206):
//     rmsnorm -> qkv gemm -> qk-norm+rope+kv-write -> attention -> o gemm (+resid)
//     -> rmsnorm -> gate/up gemm (+SwiGLU) -> down gemm (+resid)
// with no allocation and no host synchronisation on the hot path.
#include <math.h>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/inferd_span.h"
#include "common.h"
#include "kernels.h"

static thread_local std::string g_err;

static int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
int inferd_fail(int code, const std::string& msg) { return fail(code, msg); }

#define HIP_TRY(expr)                                                                      \
  do {                                                                                     \
    hipError_t _e = (expr);                                                                \
    if (_e != hipSuccess)                                                                  \
      return fail(INFERD_ERR_HIP, std::string(#expr " failed: ") + hipGetErrorString(_e)); \
  } while (0)

#define GEMM_TRY(call)                                                                      \
  do {                                                                                      \
    if (!(call)) return fail(INFERD_ERR_ARG, "internal: GEMM combination without a body"); \
  } while (0)

#define LAUNCH_CHECK()                                                                            \
  do {                                                                                            \
    hipError_t _e = hipGetLastError();                                                            \
    if (_e != hipSuccess)                                                                         \
      return fail(INFERD_ERR_HIP, std::string("kernel launch failed: ") + hipGetErrorString(_e)); \
  } while (0)

extern "C" const char* inferd_last_error(void) { return g_err.c_str(); }
extern "C" int inferd_abi_version(void) { return 5; }

namespace {

struct LayerW {
  u16* qkv = nullptr;     // packed [(H+2KV)*128][hidden]
  u16* o = nullptr;       // packed [hidden][H*128]
  u16* gateup = nullptr;  // packed [2*I][hidden]
  u16* down = nullptr;    // packed [hidden][I]
  u16* in_ln = nullptr;
  u16* post_ln = nullptr;
  u16* q_norm = nullptr;
  u16* k_norm = nullptr;
};

// tensor ids shared with oracle/weightgen.py
enum { T_Q = 0, T_K, T_V, T_O, T_QN, T_KN, T_INLN, T_POSTLN, T_GATE, T_UP, T_DOWN };
const uint32_t T_EMBED = 0xFFFF0000u, T_NORM = 0xFFFF0001u, T_LM = 0xFFFF0002u;
const float LINEAR_SCALE = 0.034641016151377546f;  // float32(0.02 * sqrt(3))
const float NORM_SCALE = 0.1f;

// kernel classes timed by inferd_span_profile_* (order = INFERD_PROF_* in the header)
enum { PROF_NORM = 0, PROF_QKV, PROF_ROPE, PROF_ATTN, PROF_O, PROF_GATEUP, PROF_DOWN, PROF_LMHEAD, PROF_NCLS };

uint64_t tensor_key(uint64_t seed, uint32_t tid) {
  return splitmix64(((seed & 0xFFFFFFFFull) << 32) | (uint64_t)tid);
}

// Decode q/k/v K-slices (reduced by the fused decode attention): the measured optimum
// (other slice counts, like every other A/B variant, live in tools/ lab
// builds -- the product library has one path per op and reads no environment).
#define QKV_KSL 2

}  // namespace

struct InferdSpan {
  InferdSpanConfig cfg;
  std::vector<LayerW> layers;
  u16* embed = nullptr;
  u16* final_norm = nullptr;
  u16* lm_head = nullptr;
  u16* cos_t = nullptr;
  u16* sin_t = nullptr;
  u16* kv_pool = nullptr;
  size_t kv_layer_elems = 0;
  // workspace
  u16 *xn = nullptr, *qkv = nullptr, *q = nullptr, *attn = nullptr, *act = nullptr, *h = nullptr,
      *last = nullptr;
  float* attn_ws = nullptr;
  size_t attn_ws_bytes = 0;
  // RMSNorms at the reference's rounding points (qwen3_server_module.py:19-25).  On the decode
  // GEMV path (<= 64 rows) the o and down GEMVs add the row sums of squares of their outputs
  // into SSQ slots (kernels.h DecodeNorm; slot 2l: layer l's o -> its gate/up, slot 2l+1: layer
  // l's down -> layer l+1's q/k/v), and those GEMVs normalise their A fragments from them; the
  // layer-0 rmsnorm_kernel zeroes the slots at the start of each such forward.  Otherwise (a
  // span's first layer, prefill) rmsnorm_kernel writes the normed rows to xn.
  unsigned long long* ssq = nullptr;
  GemmWs gws;                 // prefill tail-split workspace (per span: spans never share tickets)
  float* qkv_part = nullptr;  // decode split-K q/k/v partials [QKV_KSL][16][qkv_rows]
  unsigned long long* argmax_partial = nullptr;
  int32_t* err = nullptr;
  // set by inferd_span_graph_capture(advance): the scheduler step the next forward's first
  // RMSNorm launch runs (NormPrologue) instead of a decode_advance_kernel node of its own
  NormPrologue adv;
  bool adv_pending = false;
  std::vector<void*> allocs;
  // optional per-kernel-class timing with HIP events on the launch stream
  bool prof_on = false;
  std::vector<hipEvent_t> prof_events;
  std::vector<int> prof_class;
  size_t prof_used = 0;

  ~InferdSpan() {
    for (hipEvent_t e : prof_events) (void)hipEventDestroy(e);
    for (void* p : allocs) (void)hipFree(p);
    gemm_ws_free(&gws);
  }
  // returns the pair index or -1
  long prof_begin(int cls, hipStream_t st) {
    if (!prof_on || prof_used + 2 > prof_events.size()) return -1;
    long i = (long)prof_used;
    prof_used += 2;
    prof_class[i / 2] = cls;
    (void)hipEventRecord(prof_events[i], st);
    return i;
  }
  void prof_end(long i, hipStream_t st) {
    if (i >= 0) (void)hipEventRecord(prof_events[i + 1], st);
  }
  int alloc(void** p, size_t bytes) {
    hipError_t e = hipMalloc(p, bytes < 256 ? 256 : bytes);
    if (e != hipSuccess) {
      *p = nullptr;
      return fail(INFERD_ERR_HIP, "hipMalloc(" + std::to_string(bytes) + ") failed: " + hipGetErrorString(e));
    }
    allocs.push_back(*p);
    return INFERD_OK;
  }
  int qkv_rows() const { return (cfg.heads + 2 * cfg.kv_heads) * HEAD_DIM; }
  // the halves of span-local layer l this span runs (InferdSpanConfig skip_first_attn /
  // skip_last_mlp); only layers with an attention half own a KV pool layer
  // has_qkv: input_layernorm + q/k/v weights; has_attn: the attention kernel and a KV pool
  // layer; has_o: o_proj + residual
  bool first_no_attn() const { return cfg.skip_first_attn || cfg.o_split_first; }
  bool last_qkv_only(int l) const { return l == cfg.n_layers - 1 && cfg.qkv_split_last; }
  bool has_qkv(int l) const { return !(l == 0 && first_no_attn()); }
  bool has_attn(int l) const { return has_qkv(l) && !last_qkv_only(l); }
  bool has_o(int l) const {
    return !(l == 0 && cfg.skip_first_attn) && !(l == cfg.n_layers - 1 && cfg.o_split_last) && !last_qkv_only(l);
  }
  bool has_mlp(int l) const {
    return !(l == cfg.n_layers - 1 && (cfg.skip_last_mlp || cfg.o_split_last)) && !last_qkv_only(l);
  }
  // the last layer of a span that ends inside the layer's gate/up projection computes part of it
  bool has_gateup(int l) const { return has_mlp(l) || (l == cfg.n_layers - 1 && cfg.gateup_split_last); }
  int kv_layers() const { return cfg.n_layers - (first_no_attn() ? 1 : 0) - (cfg.qkv_split_last ? 1 : 0); }
  // the lm_head rows this span owns (InferdSpanConfig head_first / head_rows): all of them with
  // has_lm_head, else its vocab-parallel shard (0 rows: none)
  int lm_rows() const { return cfg.has_lm_head ? cfg.vocab : cfg.head_rows; }
  int lm_first() const { return cfg.has_lm_head ? 0 : cfg.head_first; }
  u16* kv_of(int l) const { return kv_pool + kv_layer_elems * (l - (first_no_attn() ? 1 : 0)); }
};

#define ALLOC(ptr, bytes)                                   \
  do {                                                      \
    int _rc = s->alloc((void**)&(ptr), (size_t)(bytes));    \
    if (_rc) return _rc;                                    \
  } while (0)

extern "C" int inferd_span_create(const InferdSpanConfig* cfg, InferdSpan** out) {
  if (!cfg || !out) return fail(INFERD_ERR_ARG, "null argument");
  const InferdSpanConfig& c = *cfg;
  if (c.head_dim != HEAD_DIM) return fail(INFERD_ERR_ARG, "head_dim must be 128");
  if ((int64_t)c.max_seqs * c.heads > 16384) return fail(INFERD_ERR_ARG, "max_seqs * heads must be <= 16384");
  if (c.kv_heads <= 0 || c.heads % c.kv_heads != 0 || c.heads / c.kv_heads > 16)
    return fail(INFERD_ERR_ARG, "heads must be a multiple of kv_heads with group size <= 16");
  if (c.hidden % 128 || c.intermediate % 64 || c.vocab % 16)
    return fail(INFERD_ERR_ARG, "hidden % 128, intermediate % 64 and vocab % 16 must be 0");
  if (c.n_layers < 0 || c.max_tokens <= 0 || c.max_seqs <= 0 || c.kv_pages <= 0 || c.max_positions <= 0)
    return fail(INFERD_ERR_ARG, "bad span sizes");
  if (c.has_lm_head && c.max_seqs > 64)
    return fail(INFERD_ERR_ARG, "a span with lm_head takes max_seqs <= 64 (the greedy argmax is per call of <= 64 rows)");
  if (c.kv_pages > (1 << 24)) return fail(INFERD_ERR_ARG, "kv_pages must be <= 2^24");
  if ((c.skip_first_attn | c.skip_last_mlp) & ~1) return fail(INFERD_ERR_ARG, "skip_first_attn / skip_last_mlp are 0 or 1");
  if (c.skip_first_attn && c.has_embed)
    return fail(INFERD_ERR_ARG, "a span with the embedding starts at a layer's attention half (skip_first_attn = 0)");
  if (c.skip_last_mlp && c.has_lm_head)
    return fail(INFERD_ERR_ARG, "a span with lm_head ends at a layer's MLP half (skip_last_mlp = 0)");
  if ((c.skip_first_attn || c.skip_last_mlp) && c.n_layers < 1)
    return fail(INFERD_ERR_ARG, "a half-layer boundary needs n_layers >= 1");
  if (c.skip_first_attn && c.skip_last_mlp && c.n_layers == 1)
    return fail(INFERD_ERR_ARG, "a one-layer span cannot skip both of its halves");
  for (int32_t col : {c.gateup_split_first, c.gateup_split_last})
    if (col < 0 || col % 128 || (col && col >= c.intermediate))
      return fail(INFERD_ERR_ARG, "gate/up split columns: 0, or a multiple of 128 below intermediate");
  if ((c.gateup_split_first && !c.skip_first_attn) || (c.gateup_split_last && !c.skip_last_mlp))
    return fail(INFERD_ERR_ARG, "a gate/up split refines a half-layer boundary (skip_first_attn / skip_last_mlp)");
  if ((c.o_split_first | c.o_split_last) & ~1) return fail(INFERD_ERR_ARG, "o_split_first / o_split_last are 0 or 1");
  if ((c.o_split_first && (c.skip_first_attn || c.has_embed)) || (c.o_split_last && (c.skip_last_mlp || c.has_lm_head)))
    return fail(INFERD_ERR_ARG, "an attention|o boundary excludes a half-layer boundary at the same end, the "
                                "embedding (first) and lm_head (last)");
  if ((c.o_split_first || c.o_split_last) && c.n_layers < 1)
    return fail(INFERD_ERR_ARG, "an attention|o boundary needs n_layers >= 1");
  if ((c.qkv_split_first | c.qkv_split_last) & ~1) return fail(INFERD_ERR_ARG, "qkv_split_first / qkv_split_last are 0 or 1");
  if ((c.qkv_split_first && (c.skip_first_attn || c.o_split_first || c.has_embed)) ||
      (c.qkv_split_last && (c.skip_last_mlp || c.o_split_last || c.has_lm_head)))
    return fail(INFERD_ERR_ARG, "a q/k/v|attention boundary excludes another sub-layer boundary at the same end, the "
                                "embedding (first) and lm_head (last)");
  if ((c.qkv_split_first || c.qkv_split_last) && c.n_layers < 1)
    return fail(INFERD_ERR_ARG, "a q/k/v|attention boundary needs n_layers >= 1");
  if (c.head_rows < 0 || c.head_first < 0 || c.head_rows % 16 || c.head_first % 16 ||
      (int64_t)c.head_first + c.head_rows > c.vocab)
    return fail(INFERD_ERR_ARG, "lm_head shard: rows [head_first, head_first + head_rows) within the vocabulary, "
                                "multiples of 16");
  if (c.final_norm_out & ~1) return fail(INFERD_ERR_ARG, "final_norm_out is 0 or 1");
  if (c.has_lm_head && (c.head_rows || c.final_norm_out))
    return fail(INFERD_ERR_ARG, "a span with the whole lm_head has no shard and no final_norm_out");
  if (c.final_norm_out && (c.skip_last_mlp || c.o_split_last || c.qkv_split_last || c.max_seqs > 64))
    return fail(INFERD_ERR_ARG, "a final_norm_out span ends at a layer boundary and takes max_seqs <= 64");
  if (c.n_layers == 1 && ((c.o_split_first && (c.o_split_last || c.skip_last_mlp)) ||
                          (c.o_split_last && c.skip_first_attn) ||
                          (c.qkv_split_last && (c.skip_first_attn || c.o_split_first || c.qkv_split_first)) ||
                          (c.qkv_split_first && c.o_split_last)))
    return fail(INFERD_ERR_ARG, "a one-layer span cannot end before the part it starts at");
  InferdSpan* s = new InferdSpan();
  s->cfg = c;
  const int h = c.hidden, I = c.intermediate, H = c.heads, KV = c.kv_heads;
  s->layers.resize(c.n_layers);
  int rc = 0;
  auto bail = [&](int code) {
    delete s;
    return code;
  };
#define SALLOC(ptr, bytes)                                  \
  do {                                                      \
    rc = s->alloc((void**)&(ptr), (size_t)(bytes));         \
    if (rc) return bail(rc);                                \
  } while (0)
  for (int l = 0; l < c.n_layers; ++l) {
    LayerW& L = s->layers[l];
    if (s->has_qkv(l)) {
      SALLOC(L.qkv, (size_t)s->qkv_rows() * h * 2);
      SALLOC(L.in_ln, (size_t)h * 2);
      SALLOC(L.q_norm, HEAD_DIM * 2);
      SALLOC(L.k_norm, HEAD_DIM * 2);
    }
    if (s->has_o(l)) SALLOC(L.o, (size_t)h * H * HEAD_DIM * 2);
    if (s->has_gateup(l)) {  // a gate/up boundary's sender owns gate/up too
      SALLOC(L.gateup, (size_t)2 * I * h * 2);
      SALLOC(L.post_ln, (size_t)h * 2);
    }
    if (s->has_mlp(l)) SALLOC(L.down, (size_t)h * I * 2);
  }
  if (c.has_embed) SALLOC(s->embed, (size_t)c.vocab * h * 2);
  if (c.has_lm_head || c.final_norm_out) SALLOC(s->final_norm, (size_t)h * 2);
  if (s->lm_rows() > 0) SALLOC(s->lm_head, (size_t)s->lm_rows() * h * 2);
  // rope tables
  SALLOC(s->cos_t, (size_t)c.max_positions * 64 * 2);
  SALLOC(s->sin_t, (size_t)c.max_positions * 64 * 2);
  {
    float inv[64];
    for (int i = 0; i < 64; ++i) {
      // HF default rope: 1 / theta ** (arange(0, d, 2) / d) evaluated in fp32 (torch pow)
      float e = (float)(2 * i) / (float)HEAD_DIM;
      inv[i] = 1.0f / powf(c.rope_theta, e);
    }
    float* dinv = nullptr;
    SALLOC(dinv, sizeof(inv));
    if (hipMemcpy(dinv, inv, sizeof(inv), hipMemcpyHostToDevice) != hipSuccess)
      return bail(fail(INFERD_ERR_HIP, "rope upload failed"));
    launch_rope_table(dinv, c.max_positions, s->cos_t, s->sin_t, 0);
  }
  // KV pool
  // whole super-pages (common.h: KV_SUPER)
  s->kv_layer_elems = (size_t)((c.kv_pages + KV_SUPER - 1) / KV_SUPER * KV_SUPER) * 2 * KV * KV_BLOCK_ELEMS;
  if (s->kv_layers() > 0) {
    SALLOC(s->kv_pool, s->kv_layer_elems * s->kv_layers() * 2);
    if (hipMemset(s->kv_pool, 0, s->kv_layer_elems * s->kv_layers() * 2) != hipSuccess)
      return bail(fail(INFERD_ERR_HIP, "kv memset failed"));
  }
  // workspace
  const size_t Mx = c.max_tokens;
  SALLOC(s->xn, ((Mx + 15) & ~(size_t)15) * h * 2);  // decode: whole packed tiles
  SALLOC(s->qkv, Mx * s->qkv_rows() * 2);
  SALLOC(s->q, Mx * H * HEAD_DIM * 2);
  SALLOC(s->attn, ((Mx + 15) & ~(size_t)15) * H * HEAD_DIM * 2);  // decode: whole packed tiles
  SALLOC(s->act, ((Mx + 15) & ~(size_t)15) * I * 2);  // decode: whole 16-row packed tiles
  SALLOC(s->h, ((Mx + 15) & ~(size_t)15) * h * 2);  // decode: whole packed tiles
  SALLOC(s->last, (((size_t)c.max_seqs + 15) & ~(size_t)15) * h * 2);  // whole packed tiles
  s->attn_ws_bytes = attn_decode_ws_bytes(c.max_seqs, H, c.max_positions);
  SALLOC(s->attn_ws, s->attn_ws_bytes);
  if (hipMemset(s->attn_ws, 0, s->attn_ws_bytes) != hipSuccess) return bail(fail(INFERD_ERR_HIP, "memset failed"));
  SALLOC(s->ssq, (size_t)(2 * c.n_layers) * SSQ_SLOT_WORDS * 8);
  if (s->lm_rows() > 0) SALLOC(s->argmax_partial, (size_t)(s->lm_rows() / 16) * 64 * 8);
  SALLOC(s->qkv_part, (size_t)QKV_KSL * 16 * s->qkv_rows() * 4);
  // the prefill tail split's workspace, once (a forward never allocates): only spans whose
  // calls can reach the 256x256 GEMMs (>= 512 rows) need it
  s->gws.split = c.max_tokens >= 512;
  if (gemm_ws_alloc(&s->gws) != (int)hipSuccess) return bail(fail(INFERD_ERR_HIP, "tail-split workspace allocation failed"));
  SALLOC(s->err, 256);
  if (hipMemset(s->err, 0, 4) != hipSuccess) return bail(fail(INFERD_ERR_HIP, "memset failed"));
  if (hipDeviceSynchronize() != hipSuccess) return bail(fail(INFERD_ERR_HIP, "init sync failed"));
  *out = s;
  return INFERD_OK;
#undef SALLOC
}

extern "C" void inferd_span_destroy(InferdSpan* span) { delete span; }

// bf16 elements of a forward / step call's x_in (which = 0) or x_out (which = 1): the hidden rows
// plus the record a sub-layer boundary carries (gate/up: the packed act over 16-row tiles in calls
// of <= 64 rows; attention|o: the attention output, 16-row tiles in pure decode calls; q/k/v|
// attention: the raw q/k/v rows in pure decode calls), or a final_norm_out span's normed last rows
// over 16-row tiles.  A pure function of the config: hosts size buffers before they create a span.
extern "C" int64_t inferd_span_io_elems(const InferdSpanConfig* c, int32_t n_tokens, int32_t n_seqs, int32_t decode,
                                        int32_t which) {
  if (!c || n_tokens < 0 || n_seqs < 0 || (which != 0 && which != 1)) {
    g_err = "inferd_span_io_elems: a config, n_tokens / n_seqs >= 0 and which 0 (x_in) or 1 (x_out)";
    return -1;
  }
  const int64_t M = n_tokens, h = c->hidden;
  const bool gemv = M <= 64;
  const int64_t rec = (M + 15) / 16 * 16 * (int64_t)c->intermediate;
  const int64_t orec = (decode && gemv ? (M + 15) / 16 * 16 : M) * (int64_t)c->heads * c->head_dim;
  const int64_t qrec = decode ? M * (int64_t)(c->heads + 2 * c->kv_heads) * c->head_dim : 0;
  if (which == 0)
    return M * h + (gemv && c->gateup_split_first ? rec : 0) + (c->o_split_first ? orec : 0) +
           (c->qkv_split_first ? qrec : 0);
  if (c->final_norm_out) return ((int64_t)n_seqs + 15) / 16 * 16 * h;
  return M * h + (gemv && c->gateup_split_last ? rec : 0) + (c->o_split_last ? orec : 0) +
         (c->qkv_split_last ? qrec : 0);
}

extern "C" int inferd_span_get_config(const InferdSpan* span, InferdSpanConfig* out) {
  if (!span || !out) return fail(INFERD_ERR_ARG, "null argument");
  *out = span->cfg;
  return INFERD_OK;
}

// ------------------------------------------------------------------ weights
namespace {
struct Target {
  u16* dst;       // destination base
  int packed;     // 1: fragment-pack at n-tile offset
  int64_t rows, cols;
  uint32_t tid_idx;
  int64_t elem0 = 0;  // generator counter of the first element (an lm_head shard: head_first * hidden)
};

int resolve_layer(InferdSpan* s, int layer, const char* name, Target* t);
bool owns_weight(const InferdSpan* s, int layer, const char* name);

int resolve(InferdSpan* s, int layer, const char* name, Target* t) {
  const InferdSpanConfig& c = s->cfg;
  const int h = c.hidden;
  if (layer < 0) {
    if (!strcmp(name, "embed_tokens") && s->embed) { *t = {s->embed, 0, c.vocab, h, T_EMBED}; return 0; }
    if (!strcmp(name, "norm") && s->final_norm) { *t = {s->final_norm, 0, 1, h, T_NORM}; return 0; }
    if (!strcmp(name, "lm_head") && s->lm_head) {
      *t = {s->lm_head, 1, s->lm_rows(), h, T_LM, (int64_t)s->lm_first() * h};
      return 0;
    }
    return fail(INFERD_ERR_ARG, std::string("unknown/unowned global weight ") + name);
  }
  if (layer >= c.n_layers) return fail(INFERD_ERR_ARG, "layer index out of span");
  if (resolve_layer(s, layer, name, t)) return INFERD_ERR_ARG;
  // by ownership, not by t->dst: a sub-tensor of an absent part (k_proj, up_proj) resolves to
  // an offset from a null base
  if (!owns_weight(s, layer, name))
    return fail(INFERD_ERR_ARG, std::string(name) + ": layer " + std::to_string(layer) +
                                    " of this span runs only its other half / part (skip_first_attn, skip_last_mlp, o_split_*, "
                                    "qkv_split_last)");
  return 0;
}

int resolve_layer(InferdSpan* s, int layer, const char* name, Target* t) {
  const InferdSpanConfig& c = s->cfg;
  const int h = c.hidden, I = c.intermediate, H = c.heads, KV = c.kv_heads;
  LayerW& L = s->layers[layer];
  const int64_t qrows = (int64_t)H * HEAD_DIM, kvrows = (int64_t)KV * HEAD_DIM;
  if (!strcmp(name, "q_proj")) { *t = {L.qkv, 1, qrows, h, T_Q}; return 0; }
  if (!strcmp(name, "k_proj")) { *t = {L.qkv + qrows * h, 1, kvrows, h, T_K}; return 0; }
  if (!strcmp(name, "v_proj")) { *t = {L.qkv + (qrows + kvrows) * h, 1, kvrows, h, T_V}; return 0; }
  if (!strcmp(name, "o_proj")) { *t = {L.o, 1, h, qrows, T_O}; return 0; }
  if (!strcmp(name, "gate_proj")) { *t = {L.gateup, 1, I, h, T_GATE}; return 0; }
  if (!strcmp(name, "up_proj")) { *t = {L.gateup + (int64_t)I * h, 1, I, h, T_UP}; return 0; }
  if (!strcmp(name, "down_proj")) { *t = {L.down, 1, h, I, T_DOWN}; return 0; }
  if (!strcmp(name, "q_norm")) { *t = {L.q_norm, 0, 1, HEAD_DIM, T_QN}; return 0; }
  if (!strcmp(name, "k_norm")) { *t = {L.k_norm, 0, 1, HEAD_DIM, T_KN}; return 0; }
  if (!strcmp(name, "input_layernorm")) { *t = {L.in_ln, 0, 1, h, T_INLN}; return 0; }
  if (!strcmp(name, "post_attention_layernorm")) { *t = {L.post_ln, 0, 1, h, T_POSTLN}; return 0; }
  return fail(INFERD_ERR_ARG, std::string("unknown layer weight ") + name);
}

// 1 if span-local layer `layer` runs the half that weight `name` belongs to
bool owns_weight(const InferdSpan* s, int layer, const char* name) {
  if (!strcmp(name, "down_proj")) return s->has_mlp(layer);
  if (!strcmp(name, "o_proj")) return s->has_o(layer);
  if (!strcmp(name, "gate_proj") || !strcmp(name, "up_proj") || !strcmp(name, "post_attention_layernorm"))
    return s->has_gateup(layer);
  return s->has_qkv(layer);
}
// packed sub-blocks start at an n-tile boundary: offset rows*K elements == (rows/16)*KT*512
}  // namespace

extern "C" int inferd_span_set_weight(InferdSpan* s, int32_t layer, const char* name,
                                      const void* src, int64_t rows, int64_t cols, void* stream) {
  if (!s || !name || !src) return fail(INFERD_ERR_ARG, "null argument");
  Target t;
  if (resolve(s, layer, name, &t)) return INFERD_ERR_ARG;
  if (rows != t.rows || cols != t.cols)
    return fail(INFERD_ERR_ARG, std::string("shape mismatch for ") + name + ": expected " +
                                    std::to_string(t.rows) + "x" + std::to_string(t.cols));
  hipStream_t st = (hipStream_t)stream;
  if (t.packed)
    launch_pack((const u16*)src, cols, (int)rows, (int)cols, t.dst, st);
  else
    HIP_TRY(hipMemcpyAsync(t.dst, src, rows * cols * 2, hipMemcpyDeviceToDevice, st));
  LAUNCH_CHECK();
  return INFERD_OK;
}

extern "C" int inferd_span_init_synthetic(InferdSpan* s, uint64_t seed, void* stream) {
  if (!s) return fail(INFERD_ERR_ARG, "null span");
  hipStream_t st = (hipStream_t)stream;
  const InferdSpanConfig& c = s->cfg;
  // temp buffer for the largest row-major tensor that needs packing
  int64_t biggest = (int64_t)c.hidden * (c.intermediate > c.heads * HEAD_DIM ? c.intermediate : c.heads * HEAD_DIM);
  if ((int64_t)s->lm_rows() * c.hidden > biggest) biggest = (int64_t)s->lm_rows() * c.hidden;
  u16* tmp = nullptr;
  HIP_TRY(hipMalloc((void**)&tmp, biggest * 2));
  static const char* layer_names[] = {"input_layernorm", "post_attention_layernorm", "q_norm", "k_norm",
                                      "q_proj", "k_proj", "v_proj", "o_proj", "gate_proj", "up_proj",
                                      "down_proj"};
  auto gen = [&](int layer, const char* name) -> int {
    Target t;
    if (resolve(s, layer, name, &t)) return INFERD_ERR_ARG;
    const bool is_norm = strstr(name, "norm") != nullptr;
    const float scale = is_norm ? NORM_SCALE : LINEAR_SCALE;
    const float center = is_norm ? 1.0f : 0.0f;
    const uint32_t tid = layer < 0 ? t.tid_idx : (uint32_t)((c.first_layer + layer) * 16 + t.tid_idx);
    const uint64_t key = tensor_key(seed, tid) + (uint64_t)t.elem0;
    const int64_t n = t.rows * t.cols;
    if (t.packed) {
      launch_weightgen(tmp, n, key, scale, center, st);
      launch_pack(tmp, t.cols, (int)t.rows, (int)t.cols, t.dst, st);
    } else {
      launch_weightgen(t.dst, n, key, scale, center, st);
    }
    return INFERD_OK;
  };
  int rc = 0;
  for (int l = 0; l < c.n_layers && !rc; ++l)
    for (const char* nm : layer_names)
      if (owns_weight(s, l, nm) && (rc = gen(l, nm))) break;
  if (!rc && c.has_embed) rc = gen(-1, "embed_tokens");
  if (!rc && s->final_norm) rc = gen(-1, "norm");
  if (!rc && s->lm_head) rc = gen(-1, "lm_head");
  hipError_t e = hipStreamSynchronize(st);
  (void)hipFree(tmp);
  if (rc) return rc;
  if (e != hipSuccess) return fail(INFERD_ERR_HIP, std::string("synthetic init: ") + hipGetErrorString(e));
  return INFERD_OK;
}

// ------------------------------------------------------------------ forward
static int check_batch(const InferdSpan* s, const InferdBatch* b) {
  const InferdSpanConfig& c = s->cfg;
  if (!b) return fail(INFERD_ERR_ARG, "null batch");
  if (b->n_tokens <= 0 || b->n_tokens > c.max_tokens)
    return fail(INFERD_ERR_ARG, "n_tokens out of range (max_tokens=" + std::to_string(c.max_tokens) + ")");
  if (b->n_seqs <= 0 || b->n_seqs > c.max_seqs) return fail(INFERD_ERR_ARG, "n_seqs out of range");
  if (b->max_ctx_len <= 0 || b->max_ctx_len > c.max_positions)
    return fail(INFERD_ERR_ARG, "max_ctx_len out of range");
  if (b->decode && b->n_tokens != b->n_seqs) return fail(INFERD_ERR_ARG, "decode batch needs one token per sequence");
  if (!b->seq_start || !b->positions || !b->ctx_lens || !b->block_table)
    return fail(INFERD_ERR_ARG, "batch arrays missing");
  if ((int64_t)b->max_pages * KV_PAGE < b->max_ctx_len) return fail(INFERD_ERR_ARG, "block table too narrow");
  return INFERD_OK;
}

// the attention's view of a batch
static AttnBatch to_attn(const InferdBatch* b) {
  AttnBatch a;
  a.seq_start = b->seq_start;
  a.positions = b->positions;
  a.ctx_lens = b->ctx_lens;
  a.block_table = b->block_table;
  a.max_pages = b->max_pages;
  a.B = b->n_seqs;
  a.M = b->n_tokens;
  a.max_q_len = b->max_q_len;
  a.max_ctx = b->max_ctx_len;
  return a;
}

extern "C" int inferd_span_forward(InferdSpan* s, const InferdBatch* b, const int32_t* ids,
                                   const void* x_in, void* x_out, int32_t* next_ids, void* logits,
                                   void* layer_out, void* stream) {
  if (!s) return fail(INFERD_ERR_ARG, "null span");
  int rc = check_batch(s, b);
  if (rc) return rc;
  const InferdSpanConfig& c = s->cfg;
  hipStream_t st = (hipStream_t)stream;
  const int M = b->n_tokens, B = b->n_seqs;
  const int h = c.hidden, I = c.intermediate, H = c.heads, KV = c.kv_heads;
  const int qkvN = s->qkv_rows();
  const float scale = 1.0f / sqrtf((float)HEAD_DIM);
  const u16* x;
  // the first RMSNorm launch (layer 0's input norm) also runs the embedding gather and a
  // pending graph scheduler step (kernels.h NormPrologue): two graph nodes fewer per step
  NormPrologue pro;
  if (s->adv_pending) {
    pro = s->adv;
    s->adv_pending = false;
  }
  // a final_norm_out span: x_out receives the final-normed last rows (below); the last layer's
  // hidden rows stay in the workspace, as on a span with lm_head
  void* const normed_out = c.final_norm_out ? x_out : nullptr;
  if (c.final_norm_out) x_out = nullptr;
  if (normed_out && B > 64) return fail(INFERD_ERR_ARG, "final_norm_out supports <= 64 sequences per call");
  if (M <= 64 && c.gateup_split_first && !x_in)
    return fail(INFERD_ERR_ARG, "a span starting inside a gate/up projection needs x_in (the hand-off record)");
  if ((c.o_split_last || c.qkv_split_last) && !x_out)
    return fail(INFERD_ERR_ARG, "a span ending before an o projection or an attention needs x_out (the hand-off record)");
  if (c.has_embed) {
    if (!ids) return fail(INFERD_ERR_ARG, "first span needs token ids");
    if (c.n_layers > 0) {
      pro.ids = ids;
      pro.table = s->embed;
      pro.vocab = c.vocab;
      pro.err = s->err;
      pro.x_out = s->h;
    } else {
      launch_embed(ids, s->embed, M, h, c.vocab, s->h, s->err, st);
    }
    x = s->h;
  } else {
    if (!x_in) return fail(INFERD_ERR_ARG, "span needs x_in hidden states");
    x = (const u16*)x_in;
  }
  if (c.n_layers == 0 && x_out && x != x_out)
    HIP_TRY(hipMemcpyAsync(x_out, x, (size_t)M * h * 2, hipMemcpyDeviceToDevice, st));
  const AttnBatch ab = to_attn(b);
  // RMSNorms (qwen3_server_module.py:19-25, :173-176): see InferdSpan::ssq_in.  gemv: every
  // projection of this call is a decode GEMV (<= 64 rows), so the o / down GEMVs can hand the
  // next norm its row sums of squares.
  const bool gemv = M <= 64;
  auto slot = [&](int i) { return s->ssq + (size_t)i * SSQ_SLOT_WORDS; };
  // decode: the residual stream between layers (and h1 inside a layer) fragment-packed
  // (common.h packed_index) for the GEMVs that read it; the input and the last layer's
  // output stay row-major, and so does every layer's output when layer_out asks for them
  const bool pkx = gemv && !layer_out && h % 128 == 0 && I % 128 == 0;
  bool x_packed = false;  // x (this layer's input) is fragment-packed
  long pe = -1;
  // decode: the attention output goes to the o projection's GEMV fragment-packed (also the
  // layout of an attention|o boundary record's second part)
  const bool pk_o = b->decode && gemv && !gemm_uses_tiled(M, h, H * HEAD_DIM, EPI_RESID);
  // a q/k/v|attention boundary: a pure decode call hands over the raw q/k/v rows behind x
  // (qkv_split_*); other calls hand over x and the receiver runs the whole layer
  const bool qrec = b->decode;
  const bool q_in = c.qkv_split_first && qrec;
  if ((c.o_split_first || q_in) && c.n_layers > 0 && (gemv || pro.positions)) {
    // a span starting at an o projection (or, decoding, at an attention) has no first RMSNorm
    // launch to carry the graph's scheduler step and the SSQ slot zeroing: a small launch of
    // its own
    launch_step_prologue(gemv ? s->ssq : nullptr, 2 * c.n_layers, M, &pro, st);
    pro = NormPrologue{};
  }
  for (int l = 0; l < c.n_layers; ++l) {
    const LayerW& W = s->layers[l];
    // the residual written by this layer's last half: x_out after the span's last layer, and
    // (row-major) the input of a last layer that ends before its o projection -- the first part
    // of the hand-off record
    u16* out = (l == c.n_layers - 1 && x_out) ? (u16*)x_out : s->h;
    bool out_packed = pkx && l < c.n_layers - 1;
    if ((c.o_split_last || c.qkv_split_last) && l == c.n_layers - 2) {
      out = (u16*)x_out;
      out_packed = false;
    }
    if (l == 0 && c.skip_first_attn) {
      // ---- a span starting at this layer's MLP half: x is h1 (row-major, the caller's), so
      // post_attention_layernorm runs as the span's first RMSNorm launch (slot zeroing and
      // the graph prologue included, like layer 0's input norm)
      pe = s->prof_begin(PROF_NORM, st);
      launch_rmsnorm(x, h, nullptr, 0, W.post_ln, s->xn, h, M, h, c.rms_eps, st, false, gemv ? s->ssq : nullptr,
                     2 * c.n_layers, &pro);
      s->prof_end(pe, st);
      const DecodeNorm dm = {DN_NONE, c.rms_eps, nullptr, nullptr};
      const int pk =
          (gemv && !gemm_uses_tiled(M, I, h, EPI_SILU) && !gemm_uses_tiled(M, h, I, EPI_RESID)) ? 1 : 0;
      // a gate/up boundary (decode): columns [0, c0) of act arrived in x_in's record behind h1;
      // this span completes the record's act in place and runs the whole down projection on it
      const int c0 = gemv ? c.gateup_split_first : 0;
      u16* actb = c0 ? (u16*)x_in + (size_t)M * h : s->act;
      pe = s->prof_begin(PROF_GATEUP, st);
      GEMM_TRY(launch_gemm(s->xn, h, W.gateup + (size_t)(c0 / 16) * (h / 32) * 512, M, I - c0, h,
                           actb + (size_t)(c0 / 32) * 512, I, nullptr, 0, EPI_SILU, nullptr, st, &s->gws, &dm, nullptr,
                           pk ? GEMM_PACK_C : 0, c0 ? I / 16 : 0));
      s->prof_end(pe, st);
      pe = s->prof_begin(PROF_DOWN, st);
      GEMM_TRY(launch_gemm(actb, I, W.down, M, h, I, out, h, x, h, EPI_RESID, nullptr, st, &s->gws, nullptr,
                           (gemv && l + 1 < c.n_layers) ? slot(2 * l + 1) : nullptr,
                           (pk ? GEMM_PACK_A : 0) | (out_packed ? GEMM_PACK_C : 0)));
      s->prof_end(pe, st);
      x = out;
      x_packed = out_packed;
      if (layer_out)
        HIP_TRY(hipMemcpyAsync((u16*)layer_out + (size_t)l * M * h, x, (size_t)M * h * 2,
                               hipMemcpyDeviceToDevice, st));
      LAUNCH_CHECK();
      continue;
    }
    // the attention output the o projection reads: this layer's, or (a span starting at an o
    // projection) the record's second part
    const u16* attn_src = s->attn;
    if (l == 0 && c.o_split_first) {  // x is the record's residual part
      attn_src = (const u16*)x_in + (size_t)M * h;
      goto o_proj;
    }
    {
    // a q/k/v|attention boundary: q_only -- this (last) layer runs its norm and q/k/v
    // projection only, into the record behind x (pure decode calls; other calls hand over x
    // alone); q_recv -- this (first) layer's q/k/v rows arrive in x_in's record
    const bool q_only = s->last_qkv_only(l);
    const bool q_recv = l == 0 && q_in;
    u16* kv_l = q_only ? nullptr : s->kv_of(l);
    u16* q_dst = q_only ? (u16*)x_out + (size_t)M * h : nullptr;
    // decode: QK-norm + RoPE + the cache write run inside the attention
    const bool fused = b->decode;
    // a span ending before this layer's o projection: the attention writes the record's second
    // part, behind the layer's input residual (row-major; copied there when it is the span's input)
    u16* attn_dst = s->attn;
    if (!s->has_o(l) && !q_only) attn_dst = (u16*)x_out + (size_t)M * h;
    // decode q/k/v K-slices (reduced inside the fused attention): M <= 16 and K/32 divisible
    // by 4 * slices
    int ksl = (fused && M <= 16) ? QKV_KSL : 1;
    if ((h / 32) % (4 * ksl)) ksl = 1;
    // ---- input_layernorm -> q/k/v projection (not on a layer whose q/k/v rows arrive in the
    // record; on a q_only layer of a call that hands over x alone, only the span's first norm
    // launch when it carries the prologue: the embedding / scheduler step)
    const u16* a_in = x;
    bool qkv_done = false;
    if (!q_recv) {
      DecodeNorm dn = {DN_NONE, c.rms_eps, nullptr, nullptr};
      if (gemv && l > 0) {
        dn = {DN_EXACT, c.rms_eps, slot(2 * l - 1), W.in_ln};
      } else if (!(q_only && !qrec && l > 0)) {
        pe = s->prof_begin(PROF_NORM, st);
        launch_rmsnorm(x, h, nullptr, 0, W.in_ln, s->xn, h, M, h, c.rms_eps, st, false, gemv ? s->ssq : nullptr,
                       2 * c.n_layers, l == 0 ? &pro : nullptr);
        s->prof_end(pe, st);
        a_in = s->xn;
      }
      if (!(q_only && !qrec)) {
        pe = s->prof_begin(PROF_QKV, st);
        // prefill: q/k norm + RoPE and the K/V cache write in the projection's epilogue when
        // the persistent GEMM runs it (else the separate qk_norm_rope_kv launch below)
        if (ksl > 1) {
          launch_gemm_decode_partial(a_in, h, W.qkv, M, qkvN, h, ksl, s->qkv_part, dn, st,
                                     (x_packed && a_in == x) ? GEMM_PACK_A : 0);
          // the record's q/k/v rows: the slices summed as the fused attention sums them
          if (q_only) launch_qkv_reduce(s->qkv_part, ksl, M, qkvN, q_dst, st);
        } else {
          if (!b->decode && !q_only) {
            const QkvEpilogue qe = {b->positions, b->slots, W.q_norm, W.k_norm, s->cos_t, s->sin_t, s->q, kv_l,
                                    H, KV, c.rms_eps};
            qkv_done = launch_gemm_qkv_fused(a_in, h, W.qkv, M, qkvN, h, qe, st);
          }
          if (!qkv_done)
            GEMM_TRY(launch_gemm(a_in, h, W.qkv, M, qkvN, h, q_only ? q_dst : s->qkv, qkvN, nullptr, 0, EPI_NONE,
                                 nullptr, st, &s->gws, &dn, nullptr, (x_packed && a_in == x) ? GEMM_PACK_A : 0));
        }
        s->prof_end(pe, st);
      }
    }
    if (q_only) {  // the record: x (first part; the span's input copied there), q/k/v rows
      if (c.n_layers == 1 && x != (const u16*)x_out)
        HIP_TRY(hipMemcpyAsync(x_out, x, (size_t)M * h * 2, hipMemcpyDeviceToDevice, st));
      LAUNCH_CHECK();
      continue;
    }
    if (fused) {  // QK-norm + RoPE + cache write inside attention
      pe = s->prof_begin(PROF_ATTN, st);
      if (q_recv)
        launch_attn_decode_fused((const u16*)x_in + (size_t)M * h, qkvN, W.q_norm, W.k_norm, s->cos_t, s->sin_t,
                                 c.rms_eps, kv_l, ab, H, KV, scale, attn_dst, s->attn_ws, st, nullptr, 0, pk_o);
      else if (ksl > 1)
        launch_attn_decode_fused(nullptr, qkvN, W.q_norm, W.k_norm, s->cos_t, s->sin_t, c.rms_eps, kv_l, ab, H, KV,
                                 scale, attn_dst, s->attn_ws, st, s->qkv_part, ksl, pk_o);
      else
        launch_attn_decode_fused(s->qkv, qkvN, W.q_norm, W.k_norm, s->cos_t, s->sin_t, c.rms_eps, kv_l, ab, H, KV,
                                 scale, attn_dst, s->attn_ws, st, nullptr, 0, pk_o);
      s->prof_end(pe, st);
    } else {
      if (!qkv_done) {
        pe = s->prof_begin(PROF_ROPE, st);
        launch_qk_norm_rope_kv(s->qkv, qkvN, b->positions, b->slots, W.q_norm, W.k_norm, s->cos_t, s->sin_t, s->q,
                               kv_l, M, H, KV, c.rms_eps, st);
        s->prof_end(pe, st);
      }
      pe = s->prof_begin(PROF_ATTN, st);
      launch_attn_prefill(s->q, kv_l, ab, H, KV, scale, attn_dst, st);
      s->prof_end(pe, st);
    }
    if (!s->has_o(l)) {  // the record: x (first part; the span's input copied there), attention output
      if (c.n_layers == 1 && x != (const u16*)x_out)
        HIP_TRY(hipMemcpyAsync(x_out, x, (size_t)M * h * 2, hipMemcpyDeviceToDevice, st));
      LAUNCH_CHECK();
      continue;
    }
    }
  o_proj:
    // ---- h1 = x + o_proj(attn)   (in place when x == s->h: same-element read-then-write)
    // h1 is packed iff pkx.  An in-place epilogue needs one layout on both sides, so h1 goes
    // to s->xn (free after the q/k/v projection) where s->h holds a row-major x (the first
    // span's embedding output) or is to receive this layer's row-major output (the last layer
    // without x_out).
    u16* h1 = (pkx && ((x == s->h && !x_packed) || (out == s->h && !out_packed))) ? s->xn : s->h;
    bool h1_packed = pkx;
    if (!s->has_mlp(l)) {
      // a span ending at this layer's attention half: h1 is the span's (row-major) output;
      // without x_out it goes to s->xn (free after the q/k/v projection), never in place over
      // a packed x
      h1 = x_out ? (u16*)x_out : s->xn;
      h1_packed = false;
      if (gemv && c.gateup_split_last && !x_out)
        return fail(INFERD_ERR_ARG, "a span ending inside a gate/up projection needs x_out (the hand-off record)");
    }
    pe = s->prof_begin(PROF_O, st);
    GEMM_TRY(launch_gemm(attn_src, H * HEAD_DIM, W.o, M, h, H * HEAD_DIM, h1, h, x, h, EPI_RESID, nullptr, st, &s->gws, nullptr,
                gemv ? slot(2 * l) : nullptr,
                (pk_o ? GEMM_PACK_A : 0) | (x_packed ? GEMM_PACK_R : 0) | (h1_packed ? GEMM_PACK_C : 0)));
    s->prof_end(pe, st);
    if (!s->has_mlp(l)) {
      const int c1 = gemv ? c.gateup_split_last : 0;
      if (c1) {
        // a gate/up boundary (decode): act columns [0, c1) go into x_out's record behind h1,
        // normed from the SSQ slot this layer's o GEMV just filled (the record's act is
        // fragment-packed with the whole projection's row length, as the receiver reads it)
        const DecodeNorm dm = {DN_EXACT, c.rms_eps, slot(2 * l), W.post_ln};
        pe = s->prof_begin(PROF_GATEUP, st);
        GEMM_TRY(launch_gemm(h1, h, W.gateup, M, c1, h, h1 + (size_t)M * h, I, nullptr, 0, EPI_SILU, nullptr, st,
                             &s->gws, &dm, nullptr, GEMM_PACK_C, I / 16));
        s->prof_end(pe, st);
      }
      x = h1;
      x_packed = false;
      if (layer_out)
        HIP_TRY(hipMemcpyAsync((u16*)layer_out + (size_t)l * M * h, x, (size_t)M * h * 2,
                               hipMemcpyDeviceToDevice, st));
      LAUNCH_CHECK();
      continue;
    }
    // ---- post_attention_layernorm -> gate/up (+SwiGLU)
    const u16* m_in = h1;
    DecodeNorm dm = {DN_NONE, c.rms_eps, nullptr, nullptr};
    if (gemv) {
      dm = {DN_EXACT, c.rms_eps, slot(2 * l), W.post_ln};
    } else {
      pe = s->prof_begin(PROF_NORM, st);
      launch_rmsnorm(h1, h, nullptr, 0, W.post_ln, s->xn, h, M, h, c.rms_eps, st);
      s->prof_end(pe, st);
      m_in = s->xn;
    }
    pe = s->prof_begin(PROF_GATEUP, st);
    // decode (the GEMV path): act goes between gate/up and down fragment-packed
    const int pk =
        (gemv && !gemm_uses_tiled(M, I, h, EPI_SILU) && !gemm_uses_tiled(M, h, I, EPI_RESID)) ? 1 : 0;
    GEMM_TRY(launch_gemm(m_in, h, W.gateup, M, I, h, s->act, I, nullptr, 0, EPI_SILU, nullptr, st, &s->gws, &dm, nullptr,
                (pk ? GEMM_PACK_C : 0) | ((pkx && m_in == h1) ? GEMM_PACK_A : 0)));
    s->prof_end(pe, st);
    // ---- x = h1 + down(act)
    pe = s->prof_begin(PROF_DOWN, st);
    GEMM_TRY(launch_gemm(s->act, I, W.down, M, h, I, out, h, h1, h, EPI_RESID, nullptr, st, &s->gws, nullptr,
                (gemv && l + 1 < c.n_layers) ? slot(2 * l + 1) : nullptr,
                (pk ? GEMM_PACK_A : 0) | (pkx ? GEMM_PACK_R : 0) | (out_packed ? GEMM_PACK_C : 0)));
    s->prof_end(pe, st);
    x = out;
    x_packed = out_packed;
    if (layer_out)
      HIP_TRY(hipMemcpyAsync((u16*)layer_out + (size_t)l * M * h, x, (size_t)M * h * 2,
                             hipMemcpyDeviceToDevice, st));
    LAUNCH_CHECK();
  }
  if (c.has_lm_head && (next_ids || logits)) {
    if (B > 64) return fail(INFERD_ERR_ARG, "lm_head argmax supports <= 64 sequences per call");
    // last row of each sequence: seq_start[b+1] - 1
    pe = s->prof_begin(PROF_LMHEAD, st);
    // the final norm writes the last rows fragment-packed for the lm_head GEMV (its A operand
    // only; the logits it may also store stay row-major).  Folding this norm into the GEMV's A
    // path (DN_EXACT, as q/k/v) measured 213.8 us in the graph against 195 + 5 us (round 3).
    const bool pk_last = h % 32 == 0;
    launch_rmsnorm(x, h, b->seq_start + 1, 1, s->final_norm, s->last, h, B, h, c.rms_eps, st, pk_last);
    GEMM_TRY(launch_gemm(s->last, h, s->lm_head, B, c.vocab, h, (u16*)logits, c.vocab, nullptr, 0, EPI_ARGMAX,
                s->argmax_partial, st, nullptr, nullptr, nullptr, pk_last ? GEMM_PACK_A : 0));
    if (next_ids) launch_argmax_reduce(s->argmax_partial, c.vocab / 16, B, next_ids, st);
    s->prof_end(pe, st);
  }
  if (normed_out) {
    // vocab-parallel head: the last row of each sequence, final-normed and fragment-packed (the
    // A operand of every stage's inferd_span_head_shard), handed over instead of running lm_head
    pe = s->prof_begin(PROF_NORM, st);
    launch_rmsnorm(x, h, b->seq_start + 1, 1, s->final_norm, (u16*)normed_out, h, B, h, c.rms_eps, st, true);
    s->prof_end(pe, st);
  }
  LAUNCH_CHECK();
  return INFERD_OK;
}

// Vocab-parallel lm_head shard: the greedy key of each row over this span's lm_head rows
// (InferdSpanConfig head_first / head_rows), column indices global.  The same GEMV and 16-column
// tiles as the whole head (inferd_span_forward's EPI_ARGMAX launch), so each logit is the one a
// single lm_head computes.
extern "C" int inferd_span_head_shard(InferdSpan* s, const void* normed, int32_t rows, const uint64_t* keys_in,
                                      uint64_t* keys_out, int32_t* ids, void* logits, void* stream) {
  if (!s || !normed || rows <= 0 || rows > 64) return fail(INFERD_ERR_ARG, "bad head_shard args (rows 1..64)");
  const InferdSpanConfig& c = s->cfg;
  const int n = s->lm_rows();
  if (n <= 0) return fail(INFERD_ERR_ARG, "span owns no lm_head rows");
  hipStream_t st = (hipStream_t)stream;
  const long pe = s->prof_begin(PROF_LMHEAD, st);
  GEMM_TRY(launch_gemm((const u16*)normed, c.hidden, s->lm_head, rows, n, c.hidden, (u16*)logits, n, nullptr, 0,
                       EPI_ARGMAX, s->argmax_partial, st, nullptr, nullptr, nullptr, GEMM_PACK_A));
  if (keys_out || ids)
    launch_argmax_keys(s->argmax_partial, n / 16, rows, s->lm_first(), (const unsigned long long*)keys_in,
                       (unsigned long long*)keys_out, ids, st);
  s->prof_end(pe, st);
  LAUNCH_CHECK();
  return INFERD_OK;
}

extern "C" int inferd_argmax_combine(const uint64_t* keys, int32_t n_parts, int32_t rows, int32_t* ids, void* stream) {
  if (!keys || !ids || n_parts <= 0 || rows <= 0) return fail(INFERD_ERR_ARG, "bad argmax_combine args");
  launch_argmax_combine((const unsigned long long*)keys, n_parts, rows, ids, (hipStream_t)stream);
  LAUNCH_CHECK();
  return INFERD_OK;
}

// Final norm + lm_head over every row of x (LastStage.forward's logits over all T positions,
// partitioned_models.py:95-96); inferd_span_forward computes them for the last rows only.
extern "C" int inferd_span_lm_head(InferdSpan* s, const void* x, int32_t rows, void* logits, void* stream) {
  if (!s || !x || !logits || rows <= 0) return fail(INFERD_ERR_ARG, "bad lm_head args");
  const InferdSpanConfig& c = s->cfg;
  if (!c.has_lm_head) return fail(INFERD_ERR_ARG, "span has no lm_head");
  if (rows > c.max_tokens) return fail(INFERD_ERR_ARG, "rows > max_tokens");
  hipStream_t st = (hipStream_t)stream;
  launch_rmsnorm((const u16*)x, c.hidden, nullptr, 0, s->final_norm, s->xn, c.hidden, rows, c.hidden, c.rms_eps, st);
  GEMM_TRY(launch_gemm(s->xn, c.hidden, s->lm_head, rows, c.vocab, c.hidden, (u16*)logits, c.vocab, nullptr, 0, EPI_NONE,
              nullptr, st, &s->gws));
  LAUNCH_CHECK();
  return INFERD_OK;
}

// ------------------------------------------------------------------ decode graphs
struct InferdGraph {
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  ~InferdGraph() {
    if (exec) (void)hipGraphExecDestroy(exec);
    if (graph) (void)hipGraphDestroy(graph);
  }
};

namespace {
// the scheduler step of a decode replay (advance) + the forward, on `st` (captured or eager)
int step_body(InferdSpan* s, const InferdBatch* b, int32_t advance, const int32_t* ids, const void* x_in, void* x_out,
              int32_t* next_ids, void* logits, hipStream_t st) {
  if (advance && s->cfg.n_layers > 0) {  // run by layer 0's input norm (NormPrologue)
    s->adv = NormPrologue{};
    s->adv.positions = (int32_t*)b->positions;
    s->adv.slots = (int32_t*)b->slots;
    s->adv.ctx_lens = (int32_t*)b->ctx_lens;
    s->adv.block_table = b->block_table;
    s->adv.max_pages = b->max_pages;
    s->adv.B = b->n_seqs;
    s->adv.err = s->err;
    s->adv_pending = true;
  } else if (advance) {
    launch_decode_advance((int32_t*)b->positions, (int32_t*)b->slots, (int32_t*)b->ctx_lens, b->block_table,
                          b->max_pages, b->n_seqs, s->err, st);
  }
  const int rc = inferd_span_forward(s, b, ids, x_in, x_out, next_ids, logits, nullptr, st);
  s->adv_pending = false;
  return rc;
}
}  // namespace

extern "C" int inferd_span_step(InferdSpan* s, const InferdBatch* b, int32_t advance, const int32_t* ids,
                                const void* x_in, void* x_out, int32_t* next_ids, void* logits, void* stream) {
  if (!s || !b) return fail(INFERD_ERR_ARG, "null argument");
  if (advance && !b->decode) return fail(INFERD_ERR_ARG, "advance needs a decode batch");
  return step_body(s, b, advance, ids, x_in, x_out, next_ids, logits, (hipStream_t)stream);
}

extern "C" int inferd_span_graph_capture(InferdSpan* s, const InferdBatch* b, int32_t advance, const int32_t* ids,
                                         const void* x_in, void* x_out, int32_t* next_ids, void* logits,
                                         void* stream, InferdGraph** out) {
  if (!s || !b || !out) return fail(INFERD_ERR_ARG, "null argument");
  if (!stream) return fail(INFERD_ERR_ARG, "graph capture needs a non-null stream");
  if (advance && !b->decode) return fail(INFERD_ERR_ARG, "advance needs a decode batch");
  hipStream_t st = (hipStream_t)stream;
  s->prof_on = false;  // event pairs are timed eagerly only (HIP cannot time captured events)
  HIP_TRY(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
  const int rc = step_body(s, b, advance, ids, x_in, x_out, next_ids, logits, st);
  hipGraph_t g = nullptr;
  hipError_t e = hipStreamEndCapture(st, &g);
  if (rc) {
    if (g) (void)hipGraphDestroy(g);
    return rc;
  }
  if (e != hipSuccess) return fail(INFERD_ERR_HIP, std::string("hipStreamEndCapture: ") + hipGetErrorString(e));
  InferdGraph* G = new InferdGraph();
  G->graph = g;
  e = hipGraphInstantiate(&G->exec, g, nullptr, nullptr, 0);
  if (e != hipSuccess) {
    delete G;
    return fail(INFERD_ERR_HIP, std::string("hipGraphInstantiate: ") + hipGetErrorString(e));
  }
  *out = G;
  return INFERD_OK;
}

extern "C" int inferd_graph_launch(InferdGraph* g, void* stream) {
  if (!g) return fail(INFERD_ERR_ARG, "null graph");
  HIP_TRY(hipGraphLaunch(g->exec, (hipStream_t)stream));
  return INFERD_OK;
}

extern "C" void inferd_graph_destroy(InferdGraph* g) { delete g; }

extern "C" int inferd_span_error_flags(InferdSpan* s, int32_t* flags) {
  if (!s || !flags) return fail(INFERD_ERR_ARG, "null argument");
  HIP_TRY(hipMemcpy(flags, s->err, 4, hipMemcpyDeviceToHost));  // synchronises the device
  if (*flags) HIP_TRY(hipMemset(s->err, 0, 4));
  return INFERD_OK;
}

extern "C" int inferd_span_profile_start(InferdSpan* s, int32_t max_pairs) {
  if (!s || max_pairs <= 0) return fail(INFERD_ERR_ARG, "bad profile args");
  while (s->prof_events.size() < (size_t)max_pairs * 2) {
    hipEvent_t e;
    HIP_TRY(hipEventCreate(&e));
    s->prof_events.push_back(e);
  }
  s->prof_class.assign(s->prof_events.size() / 2, -1);
  s->prof_used = 0;
  s->prof_on = true;
  return INFERD_OK;
}

extern "C" int inferd_span_profile_stop(InferdSpan* s, double* total_ms, int32_t* counts, int32_t n_classes) {
  if (!s) return fail(INFERD_ERR_ARG, "null span");
  s->prof_on = false;
  for (int c = 0; c < n_classes; ++c) {
    total_ms[c] = 0.0;
    counts[c] = 0;
  }
  for (size_t i = 0; i + 1 < s->prof_used; i += 2) {
    HIP_TRY(hipEventSynchronize(s->prof_events[i + 1]));
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, s->prof_events[i], s->prof_events[i + 1]));
    const int c = s->prof_class[i / 2];
    if (c >= 0 && c < n_classes) {
      total_ms[c] += ms;
      counts[c] += 1;
    }
  }
  s->prof_used = 0;
  return INFERD_OK;
}

extern "C" int inferd_span_kv_layer(InferdSpan* s, int32_t layer, void** out) {
  if (!s || !out) return fail(INFERD_ERR_ARG, "null argument");
  if (layer < 0 || layer >= s->cfg.n_layers) return fail(INFERD_ERR_ARG, "layer out of range");
  if (!s->has_attn(layer)) return fail(INFERD_ERR_ARG, "layer runs only its MLP half here (no KV)");
  *out = s->kv_of(layer);
  return INFERD_OK;
}

extern "C" int inferd_span_kv_clear(InferdSpan* s, void* stream) {
  if (!s) return fail(INFERD_ERR_ARG, "null span");
  if (s->kv_pool)
    HIP_TRY(hipMemsetAsync(s->kv_pool, 0, s->kv_layer_elems * s->kv_layers() * 2, (hipStream_t)stream));
  return INFERD_OK;
}

// ------------------------------------------------------------------ single ops
extern "C" int inferd_weightgen(void* dst, int64_t n, uint64_t seed, uint32_t tensor_id, float scale,
                                float center, void* stream) {
  if (!dst || n < 0) return fail(INFERD_ERR_ARG, "bad weightgen args");
  launch_weightgen((u16*)dst, n, tensor_key(seed, tensor_id), scale, center, (hipStream_t)stream);
  LAUNCH_CHECK();
  return INFERD_OK;
}

extern "C" int inferd_pack_weight(const void* src, int64_t rows, int64_t cols, void* dst, void* stream) {
  if (!src || !dst || rows % 16 || cols % 32) return fail(INFERD_ERR_ARG, "pack needs rows%16==0, cols%32==0");
  launch_pack((const u16*)src, cols, (int)rows, (int)cols, (u16*)dst, (hipStream_t)stream);
  LAUNCH_CHECK();
  return INFERD_OK;
}

extern "C" int inferd_unpack_weight(const void* src, int64_t rows, int64_t cols, void* dst, void* stream) {
  if (!src || !dst || rows % 16 || cols % 32) return fail(INFERD_ERR_ARG, "unpack needs rows%16==0, cols%32==0");
  launch_unpack((const u16*)src, (int)rows, (int)cols, (u16*)dst, (hipStream_t)stream);
  LAUNCH_CHECK();
  return INFERD_OK;
}

extern "C" int inferd_rmsnorm(const void* x, const void* w, void* y, int32_t rows, int32_t cols, float eps,
                              void* stream) {
  if (!x || !w || !y || rows <= 0 || cols % 8 || cols > 16384) return fail(INFERD_ERR_ARG, "bad rmsnorm args");
  launch_rmsnorm((const u16*)x, cols, nullptr, 0, (const u16*)w, (u16*)y, cols, rows, cols, eps,
                 (hipStream_t)stream);
  LAUNCH_CHECK();
  return INFERD_OK;
}

extern "C" int inferd_gemm(const void* a, const void* w, void* c, const void* r, int32_t m, int32_t n,
                           int32_t k, int32_t epi, void* stream) {
  if (!a || !w || !c || m <= 0 || n % 16 || k % 32) return fail(INFERD_ERR_ARG, "gemm needs n%16==0, k%32==0");
  if (epi < 0 || epi > 2) return fail(INFERD_ERR_ARG, "bad epilogue");
  if (epi == INFERD_EPI_RESID && !r) return fail(INFERD_ERR_ARG, "resid epilogue needs R");
  // the op API's own tail-split workspace: one per host thread, allocated on its first use and
  // freed when the thread exits (spans keep theirs)
  struct OpWs {
    GemmWs w;
    ~OpWs() { gemm_ws_free(&w); }
  };
  static thread_local OpWs op_ws;
  if (!op_ws.w.ws) {
    op_ws.w.split = 1;
    if (gemm_ws_alloc(&op_ws.w) != (int)hipSuccess) return fail(INFERD_ERR_HIP, "tail-split workspace allocation failed");
  }
  GEMM_TRY(launch_gemm((const u16*)a, k, (const u16*)w, m, n, k, (u16*)c, n, (const u16*)r, n, epi, nullptr,
              (hipStream_t)stream, &op_ws.w));
  LAUNCH_CHECK();
  return INFERD_OK;
}

extern "C" int inferd_rope_table(float theta, int32_t head_dim, int32_t max_pos, void* cos_t, void* sin_t,
                                 void* stream) {
  if (head_dim != HEAD_DIM || max_pos <= 0 || !cos_t || !sin_t) return fail(INFERD_ERR_ARG, "bad rope args");
  float inv[64];
  for (int i = 0; i < 64; ++i) inv[i] = 1.0f / powf(theta, (float)(2 * i) / (float)HEAD_DIM);
  float* dinv = nullptr;
  HIP_TRY(hipMalloc((void**)&dinv, sizeof(inv)));
  HIP_TRY(hipMemcpy(dinv, inv, sizeof(inv), hipMemcpyHostToDevice));
  launch_rope_table(dinv, max_pos, (u16*)cos_t, (u16*)sin_t, (hipStream_t)stream);
  hipError_t e = hipStreamSynchronize((hipStream_t)stream);
  (void)hipFree(dinv);
  if (e != hipSuccess) return fail(INFERD_ERR_HIP, hipGetErrorString(e));
  return INFERD_OK;
}

extern "C" int inferd_qk_norm_rope_kv(const void* qkv, const int32_t* positions, const int32_t* slots,
                                      const void* qn, const void* kn, const void* cos_t, const void* sin_t,
                                      void* q_out, void* kv_layer, int32_t m, int32_t H, int32_t KV, float eps,
                                      void* stream) {
  if (!qkv || !positions || !qn || !kn || !cos_t || !sin_t || !q_out || m <= 0 || KV <= 0 || H % KV)
    return fail(INFERD_ERR_ARG, "bad qk_norm_rope_kv args");
  if (slots && !kv_layer) return fail(INFERD_ERR_ARG, "slots given without a kv pool");
  const int ld = (H + 2 * KV) * HEAD_DIM;
  launch_qk_norm_rope_kv((const u16*)qkv, ld, positions, slots, (const u16*)qn, (const u16*)kn,
                         (const u16*)cos_t, (const u16*)sin_t, (u16*)q_out, (u16*)kv_layer, m, H, KV, eps,
                         (hipStream_t)stream);
  LAUNCH_CHECK();
  return INFERD_OK;
}

extern "C" int64_t inferd_attention_workspace_bytes(int32_t n_seqs, int32_t heads, int32_t max_ctx) {
  return (int64_t)attn_decode_ws_bytes(n_seqs, heads, max_ctx);
}

extern "C" int inferd_attention(const void* q, const void* kv_layer, const InferdBatch* b, int32_t H,
                                int32_t KV, void* out, void* ws, int64_t ws_bytes, void* stream) {
  if (!q || !kv_layer || !b || !out || KV <= 0 || H % KV || H / KV > 16) return fail(INFERD_ERR_ARG, "bad attention args");
  const AttnBatch ab = to_attn(b);
  const float scale = 1.0f / sqrtf((float)HEAD_DIM);
  if (b->decode) {
    if (!ws || ws_bytes < (int64_t)attn_decode_ws_bytes(b->n_seqs, H, b->max_ctx_len))
      return fail(INFERD_ERR_ARG, "decode attention workspace too small");
    launch_attn_decode((const u16*)q, (const u16*)kv_layer, ab, H, KV, scale, (u16*)out, (float*)ws,
                       (hipStream_t)stream);
  } else {
    launch_attn_prefill((const u16*)q, (const u16*)kv_layer, ab, H, KV, scale, (u16*)out, (hipStream_t)stream);
  }
  LAUNCH_CHECK();
  return INFERD_OK;
}
