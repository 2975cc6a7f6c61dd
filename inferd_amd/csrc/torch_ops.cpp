// PyTorch-ROCm operator registration of the span engine's C-ABI (include/inferd_span.h):
// torch.ops.inferd.* and torch.classes.inferd.DecodeGraph, the binding the node-facing host
// (inferd_amd/runtime.py) drives the engine through (BASELINE north_star: "a thin C-ABI layer
// exposed as a PyTorch-ROCm extension").  Every op is a direct
// call of extern "C" entry points of libinferd_span.so on torch's current HIP stream of the
// tensors' device; an INFERD_ERR_* status becomes a RuntimeError carrying inferd_last_error()
// (the reference's exceptions reach aiohttp the same way, partitioned_models.py:137 /
// task.py:54).  Span and page-table handles cross as int64.  Every tensor argument is checked
// against the batch shape and the span's configuration before a kernel can touch it.
// Non-torch hosts bind the same C-ABI directly (ctypes: inferd_amd/_lib.py; C:
// tests/c_abi/kv_host.c).
#include <ATen/ATen.h>
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/custom_class.h>
#include <torch/library.h>

#include <string>
#include <vector>

#include "../../include/inferd_span.h"

namespace {

void ok(int rc, const char* what) {
  TORCH_CHECK(rc == INFERD_OK, "inferd error ", rc, " in ", what, ": ", inferd_last_error());
}

template <class T>
T* handle(int64_t h, const char* what) {
  TORCH_CHECK(h != 0, what, ": null handle");
  return reinterpret_cast<T*>(h);
}

void* stream_of(at::Device d) { return (void*)c10::hip::getCurrentHIPStream(d.index()).stream(); }

const void* opt_ptr(const std::optional<at::Tensor>& t) { return t ? t->data_ptr() : nullptr; }

InferdSpanConfig config_of(InferdSpan* s) {
  InferdSpanConfig c;
  ok(inferd_span_get_config(s, &c), "span_get_config");
  return c;
}

// device, dtype, contiguity and the minimum element count of an optional tensor argument
void check_arg(const std::optional<at::Tensor>& t, at::Device dev, at::ScalarType dt, int64_t min_numel,
               const char* name) {
  if (!t) return;
  TORCH_CHECK(t->device() == dev, name, " must be on ", dev, " (is on ", t->device(), ")");
  TORCH_CHECK(t->scalar_type() == dt, name, " must be ", dt, " (is ", t->scalar_type(), ")");
  TORCH_CHECK(t->is_contiguous(), name, " must be contiguous");
  TORCH_CHECK(t->numel() >= min_numel, name, " has ", t->numel(), " elements, the call needs ", min_numel);
}

// the InferdBatch view of a device int32 descriptor [seq_start | positions | slots | ctx_lens |
// block_table] (the words inferd_kv_build_batch writes) and its shape
// [n_seqs, n_tokens, max_q_len, max_ctx_len, max_pages, decode]
InferdBatch batch_of(const at::Tensor& words, at::IntArrayRef shape) {
  TORCH_CHECK(shape.size() == 6, "batch shape: [n_seqs, n_tokens, max_q_len, max_ctx_len, max_pages, decode]");
  TORCH_CHECK(words.scalar_type() == at::kInt && words.is_contiguous() && words.is_cuda(),
              "batch words: a contiguous int32 device tensor");
  const int64_t n = shape[0], m = shape[1], mp = shape[4];
  TORCH_CHECK(n > 0 && m > 0 && mp > 0, "batch shape: empty batch");
  TORCH_CHECK(words.numel() >= n + 1 + 2 * m + n + n * mp, "batch words: too few for the shape");
  const int32_t* w = words.data_ptr<int32_t>();
  return InferdBatch{(int32_t)n, (int32_t)m, (int32_t)shape[2], (int32_t)shape[3], (int32_t)mp, (int32_t)shape[5],
                     w, w + n + 1, w + n + 1 + m, w + n + 1 + 2 * m, w + n + 1 + 2 * m + n};
}

// every buffer of one span forward over `b` against the span's sizes
void check_forward_args(const InferdSpanConfig& c, const at::Tensor& words, const InferdBatch& b,
                        const std::optional<at::Tensor>& ids, const std::optional<at::Tensor>& x,
                        const std::optional<at::Tensor>& x_out, const std::optional<at::Tensor>& next_ids,
                        const std::optional<at::Tensor>& logits, const std::optional<at::Tensor>& layers) {
  const at::Device dev = words.device();
  const int64_t M = b.n_tokens, B = b.n_seqs, h = c.hidden;
  TORCH_CHECK(!c.has_embed || ids, "a first span needs ids");
  TORCH_CHECK(c.has_embed || x, "a span without the embedding needs x");
  TORCH_CHECK(c.has_lm_head || (!next_ids && !logits), "next_ids / logits need a span with lm_head");
  check_arg(ids, dev, at::kInt, M, "ids");
  // x / x_out: the hidden rows plus a sub-layer boundary's record, or a final_norm_out span's
  // normed rows (the C-ABI's own size rule, inferd_span_io_elems)
  check_arg(x, dev, at::kBFloat16, inferd_span_io_elems(&c, (int32_t)M, (int32_t)B, b.decode, 0), "x");
  check_arg(x_out, dev, at::kBFloat16, inferd_span_io_elems(&c, (int32_t)M, (int32_t)B, b.decode, 1), "x_out");
  check_arg(next_ids, dev, at::kInt, B, "next_ids");
  check_arg(logits, dev, at::kBFloat16, B * (int64_t)c.vocab, "logits");
  check_arg(layers, dev, at::kBFloat16, (int64_t)c.n_layers * M * h, "layers");
}

// ---- span lifetime ------------------------------------------------------------------------
// cfg: [hidden, intermediate, heads, kv_heads, head_dim, vocab, first_layer, n_layers, has_embed,
//       has_lm_head, max_positions, kv_pages, max_tokens, max_seqs, skip_first_attn, skip_last_mlp,
//       gateup_split_first, gateup_split_last, o_split_first, o_split_last, qkv_split_first,
//       qkv_split_last, head_first, head_rows, final_norm_out]
// (the trailing fields may be omitted: 14 ints = whole layers, whole head)
int64_t span_create(at::IntArrayRef cfg, double rms_eps, double rope_theta, at::Device device) {
  TORCH_CHECK(cfg.size() >= 14 && cfg.size() <= 25, "span_create: 14 .. 25 config ints");
  auto opt = [&](size_t i) { return cfg.size() > i ? (int32_t)cfg[i] : 0; };
  TORCH_CHECK(device.is_cuda(), "span_create: a GPU device");
  c10::hip::HIPGuard g(device.index());
  InferdSpanConfig c{(int32_t)cfg[0], (int32_t)cfg[1], (int32_t)cfg[2], (int32_t)cfg[3], (int32_t)cfg[4],
                     (int32_t)cfg[5], (int32_t)cfg[6], (int32_t)cfg[7], (int32_t)cfg[8], (int32_t)cfg[9],
                     (float)rms_eps, (float)rope_theta, (int32_t)cfg[10], (int32_t)cfg[11], (int32_t)cfg[12],
                     (int32_t)cfg[13], opt(14), opt(15), opt(16), opt(17), opt(18), opt(19), opt(20),
                     opt(21), opt(22), opt(23), opt(24)};
  InferdSpan* s = nullptr;
  ok(inferd_span_create(&c, &s), "span_create");
  return reinterpret_cast<int64_t>(s);
}

void span_destroy(int64_t span) { inferd_span_destroy(handle<InferdSpan>(span, "span_destroy")); }

std::vector<int64_t> span_config(int64_t span) {
  const InferdSpanConfig c = config_of(handle<InferdSpan>(span, "span_config"));
  return {c.hidden, c.intermediate, c.heads, c.kv_heads, c.head_dim, c.vocab, c.first_layer, c.n_layers,
          c.has_embed, c.has_lm_head, c.max_positions, c.kv_pages, c.max_tokens, c.max_seqs,
          c.skip_first_attn, c.skip_last_mlp, c.gateup_split_first, c.gateup_split_last, c.o_split_first,
          c.o_split_last, c.qkv_split_first, c.qkv_split_last, c.head_first, c.head_rows, c.final_norm_out};
}

void span_init_synthetic(int64_t span, int64_t seed, at::Device device) {
  TORCH_CHECK(device.is_cuda(), "span_init_synthetic: a GPU device");
  c10::hip::HIPGuard g(device.index());
  ok(inferd_span_init_synthetic(handle<InferdSpan>(span, "span_init_synthetic"), (uint64_t)seed, stream_of(device)),
     "span_init_synthetic");
}

void span_set_weight(int64_t span, int64_t layer, std::string name, const at::Tensor& w) {
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kBFloat16 && w.is_contiguous(), "set_weight: contiguous bf16 GPU tensor");
  TORCH_CHECK(w.dim() == 1 || w.dim() == 2, "set_weight: a 1-D or 2-D tensor");
  c10::hip::HIPGuard g(w.device().index());
  const int64_t rows = w.dim() == 1 ? 1 : w.size(0), cols = w.dim() == 1 ? w.size(0) : w.size(1);
  // the library checks (rows, cols) against the named weight's shape
  ok(inferd_span_set_weight(handle<InferdSpan>(span, "span_set_weight"), (int32_t)layer, name.c_str(), w.data_ptr(),
                            rows, cols, stream_of(w.device())),
     "span_set_weight");
}

// sticky device error flags, read and cleared (synchronises the device)
int64_t span_error_flags(int64_t span, at::Device device) {
  TORCH_CHECK(device.is_cuda(), "span_error_flags: a GPU device");
  c10::hip::HIPGuard g(device.index());
  int32_t f = 0;
  ok(inferd_span_error_flags(handle<InferdSpan>(span, "span_error_flags"), &f), "span_error_flags");
  return f;
}

void span_profile_start(int64_t span, int64_t max_pairs) {
  ok(inferd_span_profile_start(handle<InferdSpan>(span, "span_profile_start"), (int32_t)max_pairs), "span_profile_start");
}

// per kernel class (INFERD_PROF_* order): total ms and launch counts since profile_start
std::tuple<std::vector<double>, std::vector<int64_t>> span_profile_stop(int64_t span, int64_t n_classes) {
  std::vector<double> ms(n_classes, 0.0);
  std::vector<int32_t> cnt(n_classes, 0);
  ok(inferd_span_profile_stop(handle<InferdSpan>(span, "span_profile_stop"), ms.data(), cnt.data(), (int32_t)n_classes),
     "span_profile_stop");
  return {ms, std::vector<int64_t>(cnt.begin(), cnt.end())};
}

// ---- forward -------------------------------------------------------------------------------
void span_forward(int64_t span, const at::Tensor& words, at::IntArrayRef shape, const std::optional<at::Tensor>& ids,
                  const std::optional<at::Tensor>& x, const std::optional<at::Tensor>& x_out,
                  const std::optional<at::Tensor>& next_ids, const std::optional<at::Tensor>& logits,
                  const std::optional<at::Tensor>& layers) {
  InferdSpan* s = handle<InferdSpan>(span, "span_forward");
  const InferdBatch b = batch_of(words, shape);
  check_forward_args(config_of(s), words, b, ids, x, x_out, next_ids, logits, layers);
  c10::hip::HIPGuard g(words.device().index());
  ok(inferd_span_forward(s, &b, (const int32_t*)opt_ptr(ids), opt_ptr(x), (void*)opt_ptr(x_out),
                         (int32_t*)opt_ptr(next_ids), (void*)opt_ptr(logits), (void*)opt_ptr(layers),
                         stream_of(words.device())),
     "span_forward");
}

// final norm + lm_head over every row of x [rows, hidden] -> logits [rows, vocab]
void span_lm_head(int64_t span, const at::Tensor& x, const at::Tensor& logits) {
  InferdSpan* s = handle<InferdSpan>(span, "span_lm_head");
  const InferdSpanConfig c = config_of(s);
  TORCH_CHECK(x.is_cuda(), "span_lm_head: x must be on a GPU");
  TORCH_CHECK(x.dim() == 2 && x.size(1) == c.hidden, "span_lm_head: x must be [rows, ", c.hidden, "]");
  check_arg(x, x.device(), at::kBFloat16, 0, "x");
  check_arg(logits, x.device(), at::kBFloat16, x.size(0) * (int64_t)c.vocab, "logits");
  c10::hip::HIPGuard g(x.device().index());
  ok(inferd_span_lm_head(s, x.data_ptr(), (int32_t)x.size(0), logits.data_ptr(), stream_of(x.device())), "span_lm_head");
}

// vocab-parallel lm_head: the span's shard over `rows` final-normed rows (fragment-packed, 16-row
// tiles); keys are int64 tensors holding the uint64 key bits: keys_in (the running max of the
// shards before, optional) -> keys_out = max(keys_in, this shard's) (optional, may alias), ids int32
// [rows] (optional), shard logits bf16 [rows, head rows] (optional)
void span_head_shard(int64_t span, const at::Tensor& normed, int64_t rows, const std::optional<at::Tensor>& keys_in,
                     const std::optional<at::Tensor>& keys_out, const std::optional<at::Tensor>& ids,
                     const std::optional<at::Tensor>& logits) {
  InferdSpan* s = handle<InferdSpan>(span, "span_head_shard");
  const InferdSpanConfig c = config_of(s);
  const int64_t n = c.has_lm_head ? c.vocab : c.head_rows;
  TORCH_CHECK(n > 0, "span_head_shard: the span owns no lm_head rows");
  TORCH_CHECK(rows >= 1 && rows <= 64, "span_head_shard: 1 .. 64 rows");
  TORCH_CHECK(normed.is_cuda(), "span_head_shard: normed must be on a GPU");
  const at::Device dev = normed.device();
  check_arg(normed, dev, at::kBFloat16, (rows + 15) / 16 * 16 * (int64_t)c.hidden, "normed");
  check_arg(keys_in, dev, at::kLong, rows, "keys_in");
  check_arg(keys_out, dev, at::kLong, rows, "keys_out");
  check_arg(ids, dev, at::kInt, rows, "ids");
  check_arg(logits, dev, at::kBFloat16, rows * n, "logits");
  c10::hip::HIPGuard g(dev.index());
  ok(inferd_span_head_shard(s, normed.data_ptr(), (int32_t)rows, (const uint64_t*)opt_ptr(keys_in),
                            (uint64_t*)opt_ptr(keys_out), (int32_t*)opt_ptr(ids), (void*)opt_ptr(logits),
                            stream_of(dev)),
     "span_head_shard");
}

// greedy ids from n_parts shards' keys int64 [n_parts, rows] -> ids int32 [rows]
void argmax_combine(const at::Tensor& keys, int64_t n_parts, int64_t rows, const at::Tensor& ids) {
  TORCH_CHECK(keys.is_cuda() && n_parts >= 1 && rows >= 1, "argmax_combine: GPU keys, n_parts >= 1, rows >= 1");
  const at::Device dev = keys.device();
  check_arg(keys, dev, at::kLong, n_parts * rows, "keys");
  check_arg(ids, dev, at::kInt, rows, "ids");
  c10::hip::HIPGuard g(dev.index());
  ok(inferd_argmax_combine((const uint64_t*)keys.data_ptr(), (int32_t)n_parts, (int32_t)rows, ids.data_ptr<int32_t>(),
                           stream_of(dev)),
     "argmax_combine");
}

// A compute stream with a hardware queue of its own: a CU-masked stream over every CU.  HIP maps its
// ordinary streams round-robin onto GPU_MAX_HW_QUEUES (4) hardware queues, and kernels of streams
// that share a queue run in submission order -- an RCCL receive posted ahead of its data (resident,
// waiting) would hold back every compute kernel queued behind it.  CU-masked streams get dedicated
// queues outside that pool (tools/rccl_ring_probe.py: no waiter on any pool stream blocks one).
// Returned as a hipStream_t in an int64 (torch.cuda.ExternalStream); it lives for the process.
int64_t dedicated_stream(at::Device device) {
  TORCH_CHECK(device.is_cuda(), "dedicated_stream: a GPU device");
  c10::hip::HIPGuard g(device.index());
  hipDeviceProp_t p;
  TORCH_CHECK(hipGetDeviceProperties(&p, device.index()) == hipSuccess, "dedicated_stream: device properties");
  const int n = p.multiProcessorCount;
  std::vector<uint32_t> mask((n + 31) / 32, 0xFFFFFFFFu);
  if (n % 32) mask.back() = (1u << (n % 32)) - 1;
  hipStream_t s = nullptr;
  TORCH_CHECK(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()) == hipSuccess,
              "dedicated_stream: hipExtStreamCreateWithCUMask failed");
  return reinterpret_cast<int64_t>(s);
}

// one synthetic weight tensor (the counter-based generator; oracle/weightgen.py defines the same values)
void weightgen(const at::Tensor& dst, int64_t seed, int64_t tensor_id, double scale, double center) {
  TORCH_CHECK(dst.is_cuda() && dst.scalar_type() == at::kBFloat16 && dst.is_contiguous(),
              "weightgen: contiguous bf16 GPU tensor");
  c10::hip::HIPGuard g(dst.device().index());
  ok(inferd_weightgen(dst.data_ptr(), dst.numel(), (uint64_t)seed, (uint32_t)tensor_id, (float)scale, (float)center,
                      stream_of(dst.device())),
     "weightgen");
}

// ---- KV page table (host only) -------------------------------------------------------------
int64_t kv_create(int64_t n_pages) {
  InferdKvTable* t = nullptr;
  ok(inferd_kv_create((int32_t)n_pages, &t), "kv_create");
  return reinterpret_cast<int64_t>(t);
}

void kv_destroy(int64_t table) { inferd_kv_destroy(handle<InferdKvTable>(table, "kv_destroy")); }

void kv_reserve(int64_t table, int64_t seq, int64_t n_new) {
  ok(inferd_kv_reserve(handle<InferdKvTable>(table, "kv_reserve"), (uint64_t)seq, (int32_t)n_new), "kv_reserve");
}

void kv_advance(int64_t table, at::IntArrayRef seqs, int64_t n) {
  std::vector<uint64_t> s(seqs.begin(), seqs.end());
  ok(inferd_kv_advance_many(handle<InferdKvTable>(table, "kv_advance"), s.data(), (int32_t)s.size(), (int32_t)n),
     "kv_advance");
}

void kv_release(int64_t table, int64_t seq) {
  ok(inferd_kv_release(handle<InferdKvTable>(table, "kv_release"), (uint64_t)seq), "kv_release");
}

std::tuple<int64_t, int64_t> kv_query(int64_t table, int64_t seq) {
  int32_t len = 0, np = 0;
  ok(inferd_kv_query(handle<InferdKvTable>(table, "kv_query"), (uint64_t)seq, &len, &np), "kv_query");
  return {len, np};
}

std::vector<int64_t> kv_pages(int64_t table, int64_t seq) {
  auto* t = handle<InferdKvTable>(table, "kv_pages");
  int32_t len = 0, np = 0;
  ok(inferd_kv_query(t, (uint64_t)seq, &len, &np), "kv_pages");
  std::vector<int32_t> p(np > 0 ? np : 1);
  ok(inferd_kv_pages(t, (uint64_t)seq, p.data(), np), "kv_pages");
  return std::vector<int64_t>(p.begin(), p.begin() + np);
}

int64_t kv_free_pages(int64_t table) {
  int32_t f = 0;
  ok(inferd_kv_free_pages(handle<InferdKvTable>(table, "kv_free_pages"), &f), "kv_free_pages");
  return f;
}

// the batch of `seqs` (n_new new tokens each) as (device int32 words, shape) for span_forward
std::tuple<at::Tensor, std::vector<int64_t>> kv_build_batch(int64_t table, at::IntArrayRef seqs, at::IntArrayRef n_new,
                                                            at::Device device) {
  TORCH_CHECK(seqs.size() == n_new.size() && !seqs.empty(), "kv_build_batch: one n_new per sequence");
  auto* t = handle<InferdKvTable>(table, "kv_build_batch");
  std::vector<uint64_t> s(seqs.begin(), seqs.end());
  std::vector<int32_t> nn(n_new.begin(), n_new.end());
  const int64_t words = inferd_kv_batch_words(t, s.data(), nn.data(), (int32_t)s.size());
  TORCH_CHECK(words > 0, "kv_build_batch: ", inferd_last_error());
  at::Tensor host = at::empty({words}, at::TensorOptions().dtype(at::kInt).pinned_memory(device.is_cuda()));
  at::Tensor dev = at::empty({words}, at::TensorOptions().dtype(at::kInt).device(device));
  InferdBatch b;
  ok(inferd_kv_build_batch(t, s.data(), nn.data(), (int32_t)s.size(), host.data_ptr<int32_t>(), words, dev.data_ptr(), &b),
     "kv_build_batch");
  dev.copy_(host, /*non_blocking=*/true);
  return {dev, {b.n_seqs, b.n_tokens, b.max_q_len, b.max_ctx_len, b.max_pages, b.decode}};
}

// ---- decode graphs -------------------------------------------------------------------------
// One decode step of a fixed set of sequences captured as a HIP graph (inferd_span_graph_capture
// with advance = 1; the per-token client loop of client.py:244-266 / send_message.py:46-60 as one
// replay).  The constructor reserves pages for n_steps tokens of every sequence and builds the
// descriptor natively (inferd_kv_build_decode_batch: ctx_lens = the cached lengths, max_ctx_len =
// the capacity), then captures on a side stream.  The object owns every buffer the graph's
// pointers refer to -- the descriptor and the caller's ids / x / x_out / next_ids / logits -- so
// none can be freed and reused while the graph exists.  launch() replays on the current stream
// and advances the host page table by one token (all or nothing); more than n_steps launches
// raise.  `ids` and `next_ids` may be one tensor (greedy feedback).
struct DecodeGraph : torch::CustomClassHolder {
  int64_t span = 0, table = 0, n_steps = 0, launched = 0;
  std::vector<uint64_t> seqs;
  at::Tensor words;
  std::vector<at::Tensor> keep;
  at::Device device;
  InferdGraph* graph = nullptr;
  // what launch_eager() passes to inferd_span_step (the captured replay's arguments)
  InferdBatch batch{};
  const int32_t* p_ids = nullptr;
  const void* p_x = nullptr;
  void* p_out = nullptr;
  int32_t* p_next = nullptr;
  void* p_logits = nullptr;

  DecodeGraph(int64_t span_, int64_t table_, std::vector<int64_t> seqs_, int64_t n_steps_,
              std::optional<at::Tensor> ids, std::optional<at::Tensor> x, std::optional<at::Tensor> x_out,
              std::optional<at::Tensor> next_ids, std::optional<at::Tensor> logits, at::Device device_)
      : span(span_), table(table_), n_steps(n_steps_), device(device_) {
    TORCH_CHECK(device.is_cuda(), "DecodeGraph: a GPU device");
    TORCH_CHECK(!seqs_.empty() && n_steps > 0, "DecodeGraph: sequences and n_steps >= 1");
    InferdSpan* s = handle<InferdSpan>(span, "DecodeGraph");
    auto* t = handle<InferdKvTable>(table, "DecodeGraph");
    seqs.assign(seqs_.begin(), seqs_.end());
    const int32_t n = (int32_t)seqs.size();
    const int64_t nw = inferd_kv_decode_batch_words(t, seqs.data(), n, (int32_t)n_steps);
    TORCH_CHECK(nw > 0, "DecodeGraph: ", inferd_last_error());
    at::Tensor host = at::empty({nw}, at::TensorOptions().dtype(at::kInt));
    words = at::empty({nw}, at::TensorOptions().dtype(at::kInt).device(device));
    InferdBatch b;
    ok(inferd_kv_build_decode_batch(t, seqs.data(), n, (int32_t)n_steps, host.data_ptr<int32_t>(), nw, words.data_ptr(),
                                    &b),
       "DecodeGraph: kv_build_decode_batch");
    c10::hip::HIPGuard g(device.index());
    words.copy_(host);
    check_forward_args(config_of(s), words, b, ids, x, x_out, next_ids, logits, std::nullopt);
    for (const auto* o : {&ids, &x, &x_out, &next_ids, &logits})
      if (*o) keep.push_back(**o);
    // capture on a side stream (the legacy default stream cannot capture), ordered after the
    // current stream's work and before its later work
    c10::hip::HIPStream cs = c10::hip::getStreamFromPool(false, device.index());
    hipStream_t cur = c10::hip::getCurrentHIPStream(device.index()).stream();
    hipEvent_t ev;
    TORCH_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess, "DecodeGraph: event");
    (void)hipEventRecord(ev, cur);
    (void)hipStreamWaitEvent(cs.stream(), ev, 0);
    const int rc = inferd_span_graph_capture(s, &b, 1, (const int32_t*)opt_ptr(ids), opt_ptr(x), (void*)opt_ptr(x_out),
                                             (int32_t*)opt_ptr(next_ids), (void*)opt_ptr(logits), (void*)cs.stream(),
                                             &graph);
    (void)hipEventRecord(ev, cs.stream());
    (void)hipStreamWaitEvent(cur, ev, 0);
    (void)hipEventDestroy(ev);
    ok(rc, "DecodeGraph: graph_capture");
    batch = b;
    p_ids = (const int32_t*)opt_ptr(ids);
    p_x = opt_ptr(x);
    p_out = (void*)opt_ptr(x_out);
    p_next = (int32_t*)opt_ptr(next_ids);
    p_logits = (void*)opt_ptr(logits);
  }
  ~DecodeGraph() override {
    if (graph) inferd_graph_destroy(graph);
  }
  void launch() {
    TORCH_CHECK(launched < n_steps, "decode graph ran out of reserved steps (", n_steps, ")");
    c10::hip::HIPGuard g(device.index());
    ok(inferd_graph_launch(graph, stream_of(device)), "DecodeGraph.launch");
    ++launched;
    // the host page table follows the device-side advance: one native call per replay
    ok(inferd_kv_advance_many(handle<InferdKvTable>(table, "DecodeGraph"), seqs.data(), (int32_t)seqs.size(), 1),
       "DecodeGraph.launch: kv_advance");
  }
  // the same step launched kernel by kernel (no graph: no per-replay graph launch cost on the GPU)
  void launch_eager() {
    TORCH_CHECK(launched < n_steps, "decode graph ran out of reserved steps (", n_steps, ")");
    c10::hip::HIPGuard g(device.index());
    ok(inferd_span_step(handle<InferdSpan>(span, "DecodeGraph"), &batch, 1, p_ids, p_x, p_out, p_next, p_logits,
                        stream_of(device)),
       "DecodeGraph.launch_eager");
    ++launched;
    ok(inferd_kv_advance_many(handle<InferdKvTable>(table, "DecodeGraph"), seqs.data(), (int32_t)seqs.size(), 1),
       "DecodeGraph.launch_eager: kv_advance");
  }
  int64_t steps_left() const { return n_steps - launched; }
};

}  // namespace

TORCH_LIBRARY(inferd, m) {
  m.def("span_create(int[] cfg, float rms_eps, float rope_theta, Device device) -> int", &span_create);
  m.def("span_destroy(int span) -> ()", &span_destroy);
  m.def("span_config(int span) -> int[]", &span_config);
  m.def("span_init_synthetic(int span, int seed, Device device) -> ()", &span_init_synthetic);
  m.def("span_set_weight(int span, int layer, str name, Tensor w) -> ()", &span_set_weight);
  m.def("span_error_flags(int span, Device device) -> int", &span_error_flags);
  m.def("span_profile_start(int span, int max_pairs) -> ()", &span_profile_start);
  m.def("span_profile_stop(int span, int n_classes) -> (float[], int[])", &span_profile_stop);
  m.def("span_forward(int span, Tensor words, int[] shape, Tensor? ids, Tensor? x, Tensor(a!)? x_out, "
        "Tensor(b!)? next_ids, Tensor(c!)? logits, Tensor(d!)? layers=None) -> ()",
        &span_forward);
  m.def("span_lm_head(int span, Tensor x, Tensor(a!) logits) -> ()", &span_lm_head);
  m.def("span_head_shard(int span, Tensor normed, int rows, Tensor? keys_in, Tensor(a!)? keys_out, "
        "Tensor(b!)? ids, Tensor(c!)? logits=None) -> ()",
        &span_head_shard);
  m.def("argmax_combine(Tensor keys, int n_parts, int rows, Tensor(a!) ids) -> ()", &argmax_combine);
  m.def("dedicated_stream(Device device) -> int", &dedicated_stream);
  m.def("weightgen(Tensor(a!) dst, int seed, int tensor_id, float scale, float center) -> ()", &weightgen);
  m.def("kv_create(int n_pages) -> int", &kv_create);
  m.def("kv_destroy(int table) -> ()", &kv_destroy);
  m.def("kv_reserve(int table, int seq, int n_new) -> ()", &kv_reserve);
  m.def("kv_advance(int table, int[] seqs, int n) -> ()", &kv_advance);
  m.def("kv_release(int table, int seq) -> ()", &kv_release);
  m.def("kv_query(int table, int seq) -> (int, int)", &kv_query);
  m.def("kv_pages(int table, int seq) -> int[]", &kv_pages);
  m.def("kv_free_pages(int table) -> int", &kv_free_pages);
  m.def("kv_build_batch(int table, int[] seqs, int[] n_new, Device device) -> (Tensor, int[])", &kv_build_batch);
  m.class_<DecodeGraph>("DecodeGraph")
      .def(torch::init<int64_t, int64_t, std::vector<int64_t>, int64_t, std::optional<at::Tensor>,
                       std::optional<at::Tensor>, std::optional<at::Tensor>, std::optional<at::Tensor>,
                       std::optional<at::Tensor>, at::Device>())
      .def("launch", &DecodeGraph::launch)
      .def("launch_eager", &DecodeGraph::launch_eager)
      .def("steps_left", &DecodeGraph::steps_left);
}
