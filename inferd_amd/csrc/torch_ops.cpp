// PyTorch-ROCm operator registration of the span engine's C-ABI (include/inferd_span.h):
// torch.ops.inferd.* for torch hosts (BASELINE north_star: "a thin C-ABI layer exposed as a
// PyTorch-ROCm extension").  Every op is a direct call of one
// extern "C" entry point of libinferd_span.so on torch's current HIP stream of the tensors'
// device; an INFERD_ERR_* status becomes a RuntimeError carrying inferd_last_error() (the
// reference's exceptions reach aiohttp the same way, partitioned_models.py:137 / task.py:54).
// Handles (InferdSpan*, InferdKvTable*, InferdGraph*) cross as int64.  Non-torch hosts bind the
// same C-ABI directly (ctypes: inferd_amd/_lib.py; C: tests/c_abi/kv_host.c).
#include <ATen/ATen.h>
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>
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

void* stream_of(const at::Tensor& t) { return (void*)c10::hip::getCurrentHIPStream(t.device().index()).stream(); }

const void* opt_ptr(const std::optional<at::Tensor>& t) { return t ? t->data_ptr() : nullptr; }

void check_dev(const std::optional<at::Tensor>& t, const at::Tensor& ref, at::ScalarType dt, const char* name) {
  if (!t) return;
  TORCH_CHECK(t->device() == ref.device(), name, " must be on ", ref.device());
  TORCH_CHECK(t->scalar_type() == dt, name, " has the wrong dtype");
  TORCH_CHECK(t->is_contiguous(), name, " must be contiguous");
}

// the InferdBatch view of a device int32 descriptor [seq_start | positions | slots | ctx_lens |
// block_table] (the words inferd_kv_build_batch writes) and its shape
// [n_seqs, n_tokens, max_q_len, max_ctx_len, max_pages, decode]
InferdBatch batch_of(const at::Tensor& words, at::IntArrayRef shape) {
  TORCH_CHECK(shape.size() == 6, "batch shape: [n_seqs, n_tokens, max_q_len, max_ctx_len, max_pages, decode]");
  TORCH_CHECK(words.scalar_type() == at::kInt && words.is_contiguous() && words.is_cuda(),
              "batch words: a contiguous int32 device tensor");
  const int64_t n = shape[0], m = shape[1], mp = shape[4];
  TORCH_CHECK(words.numel() >= n + 1 + 2 * m + n + n * mp, "batch words: too few for the shape");
  const int32_t* w = words.data_ptr<int32_t>();
  return InferdBatch{(int32_t)n, (int32_t)m, (int32_t)shape[2], (int32_t)shape[3], (int32_t)mp, (int32_t)shape[5],
                     w, w + n + 1, w + n + 1 + m, w + n + 1 + 2 * m, w + n + 1 + 2 * m + n};
}

// ---- span lifetime ------------------------------------------------------------------------
// cfg: [hidden, intermediate, heads, kv_heads, head_dim, vocab, first_layer, n_layers, has_embed,
//       has_lm_head, max_positions, kv_pages, max_tokens, max_seqs]
int64_t span_create(at::IntArrayRef cfg, double rms_eps, double rope_theta, at::Device device) {
  TORCH_CHECK(cfg.size() == 14, "span_create: 14 config ints");
  TORCH_CHECK(device.is_cuda(), "span_create: a GPU device");
  c10::hip::HIPGuard g(device.index());
  InferdSpanConfig c{(int32_t)cfg[0], (int32_t)cfg[1], (int32_t)cfg[2], (int32_t)cfg[3], (int32_t)cfg[4],
                     (int32_t)cfg[5], (int32_t)cfg[6], (int32_t)cfg[7], (int32_t)cfg[8], (int32_t)cfg[9],
                     (float)rms_eps, (float)rope_theta, (int32_t)cfg[10], (int32_t)cfg[11], (int32_t)cfg[12],
                     (int32_t)cfg[13]};
  InferdSpan* s = nullptr;
  ok(inferd_span_create(&c, &s), "span_create");
  return reinterpret_cast<int64_t>(s);
}

void span_destroy(int64_t span) { inferd_span_destroy(handle<InferdSpan>(span, "span_destroy")); }

void span_init_synthetic(int64_t span, int64_t seed, at::Device device) {
  c10::hip::HIPGuard g(device.index());
  ok(inferd_span_init_synthetic(handle<InferdSpan>(span, "span_init_synthetic"), (uint64_t)seed,
                                (void*)c10::hip::getCurrentHIPStream(device.index()).stream()),
     "span_init_synthetic");
}

void span_set_weight(int64_t span, int64_t layer, std::string name, const at::Tensor& w) {
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kBFloat16 && w.is_contiguous(), "set_weight: contiguous bf16 GPU tensor");
  c10::hip::HIPGuard g(w.device().index());
  const int64_t rows = w.dim() == 1 ? 1 : w.size(0), cols = w.dim() == 1 ? w.size(0) : w.size(1);
  ok(inferd_span_set_weight(handle<InferdSpan>(span, "span_set_weight"), (int32_t)layer, name.c_str(), w.data_ptr(),
                            rows, cols, stream_of(w)),
     "span_set_weight");
}

// ---- forward -------------------------------------------------------------------------------
void span_forward(int64_t span, const at::Tensor& words, at::IntArrayRef shape, const std::optional<at::Tensor>& ids,
                  const std::optional<at::Tensor>& x, const std::optional<at::Tensor>& x_out,
                  const std::optional<at::Tensor>& next_ids, const std::optional<at::Tensor>& logits) {
  check_dev(ids, words, at::kInt, "ids");
  check_dev(x, words, at::kBFloat16, "x");
  check_dev(x_out, words, at::kBFloat16, "x_out");
  check_dev(next_ids, words, at::kInt, "next_ids");
  check_dev(logits, words, at::kBFloat16, "logits");
  c10::hip::HIPGuard g(words.device().index());
  const InferdBatch b = batch_of(words, shape);
  ok(inferd_span_forward(handle<InferdSpan>(span, "span_forward"), &b, (const int32_t*)opt_ptr(ids), opt_ptr(x),
                         (void*)opt_ptr(x_out), (int32_t*)opt_ptr(next_ids), (void*)opt_ptr(logits), nullptr,
                         stream_of(words)),
     "span_forward");
}

void span_lm_head(int64_t span, const at::Tensor& x, const at::Tensor& logits) {
  check_dev(logits, x, at::kBFloat16, "logits");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && x.is_contiguous(), "x: contiguous bf16");
  c10::hip::HIPGuard g(x.device().index());
  ok(inferd_span_lm_head(handle<InferdSpan>(span, "span_lm_head"), x.data_ptr(), (int32_t)x.size(0), logits.data_ptr(),
                         stream_of(x)),
     "span_lm_head");
}

// decode graphs: capture with the device-side scheduler step (advance = 1), replay, destroy
int64_t graph_capture(int64_t span, const at::Tensor& words, at::IntArrayRef shape, const std::optional<at::Tensor>& ids,
                      const std::optional<at::Tensor>& x, const std::optional<at::Tensor>& x_out,
                      const std::optional<at::Tensor>& next_ids, const std::optional<at::Tensor>& logits) {
  c10::hip::HIPGuard g(words.device().index());
  const InferdBatch b = batch_of(words, shape);
  // capture on a side stream (the legacy default stream cannot capture)
  c10::hip::HIPStream cs = c10::hip::getStreamFromPool(false, words.device().index());
  hipStream_t cur = c10::hip::getCurrentHIPStream(words.device().index()).stream();
  hipEvent_t ev;
  TORCH_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess, "graph_capture: event");
  (void)hipEventRecord(ev, cur);
  (void)hipStreamWaitEvent(cs.stream(), ev, 0);
  InferdGraph* gr = nullptr;
  const int rc = inferd_span_graph_capture(handle<InferdSpan>(span, "graph_capture"), &b, 1,
                                           (const int32_t*)opt_ptr(ids), opt_ptr(x), (void*)opt_ptr(x_out),
                                           (int32_t*)opt_ptr(next_ids), (void*)opt_ptr(logits), (void*)cs.stream(), &gr);
  (void)hipEventRecord(ev, cs.stream());
  (void)hipStreamWaitEvent(cur, ev, 0);
  (void)hipEventDestroy(ev);
  ok(rc, "graph_capture");
  return reinterpret_cast<int64_t>(gr);
}

void graph_launch(int64_t graph, at::Device device) {
  c10::hip::HIPGuard g(device.index());
  ok(inferd_graph_launch(handle<InferdGraph>(graph, "graph_launch"),
                         (void*)c10::hip::getCurrentHIPStream(device.index()).stream()),
     "graph_launch");
}

void graph_destroy(int64_t graph) { inferd_graph_destroy(handle<InferdGraph>(graph, "graph_destroy")); }

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

}  // namespace

TORCH_LIBRARY(inferd, m) {
  m.def("span_create(int[] cfg, float rms_eps, float rope_theta, Device device) -> int", &span_create);
  m.def("span_destroy(int span) -> ()", &span_destroy);
  m.def("span_init_synthetic(int span, int seed, Device device) -> ()", &span_init_synthetic);
  m.def("span_set_weight(int span, int layer, str name, Tensor w) -> ()", &span_set_weight);
  m.def("span_forward(int span, Tensor words, int[] shape, Tensor? ids, Tensor? x, Tensor(a!)? x_out, "
        "Tensor(b!)? next_ids, Tensor(c!)? logits) -> ()",
        &span_forward);
  m.def("span_lm_head(int span, Tensor x, Tensor(a!) logits) -> ()", &span_lm_head);
  m.def("graph_capture(int span, Tensor words, int[] shape, Tensor? ids, Tensor? x, Tensor(a!)? x_out, "
        "Tensor(b!)? next_ids, Tensor(c!)? logits) -> int",
        &graph_capture);
  m.def("graph_launch(int graph, Device device) -> ()", &graph_launch);
  m.def("graph_destroy(int graph) -> ()", &graph_destroy);
  m.def("kv_create(int n_pages) -> int", &kv_create);
  m.def("kv_destroy(int table) -> ()", &kv_destroy);
  m.def("kv_reserve(int table, int seq, int n_new) -> ()", &kv_reserve);
  m.def("kv_advance(int table, int[] seqs, int n) -> ()", &kv_advance);
  m.def("kv_release(int table, int seq) -> ()", &kv_release);
  m.def("kv_query(int table, int seq) -> (int, int)", &kv_query);
  m.def("kv_build_batch(int table, int[] seqs, int[] n_new, Device device) -> (Tensor, int[])", &kv_build_batch);
}
