// Host-side KV page table behind the C-ABI (include/inferd_span.h, "KV page table"): the
// per-sequence page lists and cached lengths a span's paged KV pool is addressed by, and the
// batch descriptor (InferdBatch's int32 arrays) a forward call reads.  It replaces the
// reference's per-session DynamicCache bookkeeping (qwen3_server_module.py:220,253: one
// cache per session id, appended to by every send) and the position arithmetic of
// partitioned_models.py:139-143 (positions 0..T-1 of a stateless recompute) and
// client.py:244-266 (cache_position = past .. past + T - 1 of a cached step).
//
// Pages are handed out lowest id first and a released sequence's pages go back in order, so
// a fixed sequence of calls always yields the same page ids (and the same slots).
// No device calls: a non-Python host builds its batches with these entry points and copies
// the int32 words to the device itself.
#include <algorithm>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/inferd_span.h"
#include "kernels.h"

struct InferdKvTable {
  int32_t n_pages = 0;
  std::vector<int32_t> free;  // stack: back() is the next page handed out
  struct Seq {
    std::vector<int32_t> pages;
    int32_t length = 0;  // tokens already in the cache
  };
  std::unordered_map<uint64_t, Seq> seqs;
};

namespace {

constexpr int32_t P = INFERD_KV_PAGE_TOKENS;

int32_t pages_for(int64_t tokens) { return (int32_t)((tokens + P - 1) / P); }

// validates a batch request; on success fills the descriptor's shape
int batch_shape(const InferdKvTable* t, const uint64_t* seqs, const int32_t* n_new, int32_t n, int64_t* tokens,
                int32_t* max_pages) {
  if (!t || n <= 0 || !seqs || !n_new) return inferd_fail(INFERD_ERR_ARG, "kv batch: empty request list");
  int64_t m = 0;
  int32_t mp = 1;
  for (int32_t i = 0; i < n; ++i) {
    auto it = t->seqs.find(seqs[i]);
    if (it == t->seqs.end()) return inferd_fail(INFERD_ERR_ARG, "kv batch: sequence not reserved");
    if (n_new[i] <= 0) return inferd_fail(INFERD_ERR_ARG, "kv batch: a sequence needs >= 1 new token");
    if ((int64_t)it->second.pages.size() * P < (int64_t)it->second.length + n_new[i])
      return inferd_fail(INFERD_ERR_ARG, "kv batch: pages not reserved for the new tokens");
    for (int32_t j = 0; j < i; ++j)
      if (seqs[j] == seqs[i]) return inferd_fail(INFERD_ERR_ARG, "kv batch: a sequence may appear only once");
    m += n_new[i];
    mp = std::max(mp, (int32_t)it->second.pages.size());
  }
  *tokens = m;
  *max_pages = mp;
  return INFERD_OK;
}

}  // namespace

extern "C" int inferd_kv_create(int32_t n_pages, InferdKvTable** out) {
  if (!out || n_pages <= 0) return inferd_fail(INFERD_ERR_ARG, "kv_create: n_pages must be > 0");
  auto* t = new InferdKvTable;
  t->n_pages = n_pages;
  t->free.resize(n_pages);
  for (int32_t i = 0; i < n_pages; ++i) t->free[i] = n_pages - 1 - i;
  *out = t;
  return INFERD_OK;
}

extern "C" void inferd_kv_destroy(InferdKvTable* t) { delete t; }

extern "C" int inferd_kv_reserve(InferdKvTable* t, uint64_t seq, int32_t n_new) {
  if (!t || n_new < 0) return inferd_fail(INFERD_ERR_ARG, "kv_reserve: bad argument");
  auto it = t->seqs.find(seq);
  const int32_t have = it == t->seqs.end() ? 0 : (int32_t)it->second.pages.size();
  const int32_t len = it == t->seqs.end() ? 0 : it->second.length;
  const int32_t need = pages_for((int64_t)len + n_new) - have;
  if (need > (int32_t)t->free.size())
    return inferd_fail(INFERD_ERR_NOMEM, "KV pool exhausted: need " + std::to_string(need) + " pages, " +
                                             std::to_string(t->free.size()) + " free of " +
                                             std::to_string(t->n_pages));
  auto& s = t->seqs[seq];
  for (int32_t i = 0; i < need; ++i) {
    s.pages.push_back(t->free.back());
    t->free.pop_back();
  }
  return INFERD_OK;
}

extern "C" int inferd_kv_advance(InferdKvTable* t, uint64_t seq, int32_t n) {
  if (!t || n < 0) return inferd_fail(INFERD_ERR_ARG, "kv_advance: bad argument");
  auto it = t->seqs.find(seq);
  if (it == t->seqs.end()) return inferd_fail(INFERD_ERR_ARG, "kv_advance: sequence not reserved");
  if ((int64_t)it->second.length + n > (int64_t)it->second.pages.size() * P)
    return inferd_fail(INFERD_ERR_ARG, "kv_advance: past the reserved pages");
  it->second.length += n;
  return INFERD_OK;
}

extern "C" int inferd_kv_advance_many(InferdKvTable* t, const uint64_t* seqs, int32_t n_seqs, int32_t n) {
  if (!t || n < 0 || n_seqs < 0 || (n_seqs > 0 && !seqs)) return inferd_fail(INFERD_ERR_ARG, "kv_advance_many: bad argument");
  std::vector<InferdKvTable::Seq*> ss(n_seqs);
  for (int32_t i = 0; i < n_seqs; ++i) {  // validate all first: all or nothing
    auto it = t->seqs.find(seqs[i]);
    if (it == t->seqs.end()) return inferd_fail(INFERD_ERR_ARG, "kv_advance_many: sequence not reserved");
    if ((int64_t)it->second.length + n > (int64_t)it->second.pages.size() * P)
      return inferd_fail(INFERD_ERR_ARG, "kv_advance_many: past the reserved pages");
    for (int32_t j = 0; j < i; ++j)
      if (ss[j] == &it->second) return inferd_fail(INFERD_ERR_ARG, "kv_advance_many: a sequence may appear only once");
    ss[i] = &it->second;
  }
  for (auto* q : ss) q->length += n;
  return INFERD_OK;
}

extern "C" int inferd_kv_release(InferdKvTable* t, uint64_t seq) {
  if (!t) return inferd_fail(INFERD_ERR_ARG, "kv_release: null table");
  auto it = t->seqs.find(seq);
  if (it == t->seqs.end()) return INFERD_OK;
  const auto& pg = it->second.pages;
  for (auto p = pg.rbegin(); p != pg.rend(); ++p) t->free.push_back(*p);
  t->seqs.erase(it);
  return INFERD_OK;
}

extern "C" int inferd_kv_query(const InferdKvTable* t, uint64_t seq, int32_t* length, int32_t* n_pages) {
  if (!t || !length || !n_pages) return inferd_fail(INFERD_ERR_ARG, "kv_query: bad argument");
  auto it = t->seqs.find(seq);
  *length = it == t->seqs.end() ? -1 : it->second.length;
  *n_pages = it == t->seqs.end() ? 0 : (int32_t)it->second.pages.size();
  return INFERD_OK;
}

extern "C" int inferd_kv_pages(const InferdKvTable* t, uint64_t seq, int32_t* pages, int32_t cap) {
  if (!t || (!pages && cap > 0)) return inferd_fail(INFERD_ERR_ARG, "kv_pages: bad argument");
  auto it = t->seqs.find(seq);
  if (it == t->seqs.end()) return inferd_fail(INFERD_ERR_ARG, "kv_pages: sequence not reserved");
  if ((int32_t)it->second.pages.size() > cap) return inferd_fail(INFERD_ERR_ARG, "kv_pages: buffer too small");
  std::copy(it->second.pages.begin(), it->second.pages.end(), pages);
  return INFERD_OK;
}

extern "C" int inferd_kv_free_pages(const InferdKvTable* t, int32_t* n_free) {
  if (!t || !n_free) return inferd_fail(INFERD_ERR_ARG, "kv_free_pages: bad argument");
  *n_free = (int32_t)t->free.size();
  return INFERD_OK;
}

extern "C" int64_t inferd_kv_batch_words(const InferdKvTable* t, const uint64_t* seqs, const int32_t* n_new,
                                         int32_t n) {
  int64_t m;
  int32_t mp;
  if (batch_shape(t, seqs, n_new, n, &m, &mp) != INFERD_OK) return -1;
  return (int64_t)n + 1 + 2 * m + n + (int64_t)n * mp;
}

extern "C" int inferd_kv_build_batch(const InferdKvTable* t, const uint64_t* seqs, const int32_t* n_new, int32_t n,
                                     int32_t* host, int64_t words, const void* device_base, InferdBatch* out) {
  int64_t m;
  int32_t mp;
  if (int rc = batch_shape(t, seqs, n_new, n, &m, &mp); rc != INFERD_OK) return rc;
  const int64_t need = (int64_t)n + 1 + 2 * m + n + (int64_t)n * mp;
  if (!host || !out || words < need) return inferd_fail(INFERD_ERR_ARG, "kv_build_batch: host buffer too small");
  if (m > INT32_MAX) return inferd_fail(INFERD_ERR_ARG, "kv_build_batch: too many tokens");
  // [seq_start n+1 | positions m | slots m | ctx_lens n | block_table n x mp]
  int32_t* seq_start = host;
  int32_t* pos = seq_start + n + 1;
  int32_t* slots = pos + m;
  int32_t* ctx = slots + m;
  int32_t* table = ctx + n;
  std::fill(table, table + (int64_t)n * mp, 0);
  int32_t o = 0, max_q = 0, max_ctx = 0;
  bool decode = true;
  for (int32_t i = 0; i < n; ++i) {
    const auto& s = t->seqs.at(seqs[i]);
    seq_start[i] = o;
    for (int32_t k = 0; k < n_new[i]; ++k) {
      const int32_t p = s.length + k;
      pos[o + k] = p;
      slots[o + k] = s.pages[p / P] * P + p % P;
    }
    ctx[i] = s.length + n_new[i];
    std::copy(s.pages.begin(), s.pages.end(), table + (int64_t)i * mp);
    o += n_new[i];
    max_q = std::max(max_q, n_new[i]);
    max_ctx = std::max(max_ctx, ctx[i]);
    decode = decode && n_new[i] == 1;
  }
  seq_start[n] = o;
  const int32_t* base = (const int32_t*)device_base;
  *out = InferdBatch{n, (int32_t)m, max_q, max_ctx, mp, decode ? 1 : 0, base, base + (n + 1), base + (n + 1 + m),
                     base + (n + 1 + 2 * m), base + (n + 1 + 2 * m + n)};
  return INFERD_OK;
}

// The decode-graph descriptor (inferd_span_graph_capture with advance = 1): every sequence gets
// pages for n_steps more tokens (all or nothing), positions and slots start at 0 (the graph's
// device-side scheduler step writes them before each replay), ctx_lens = the cached lengths
// and max_ctx_len = the capacity, max(length) + n_steps.
namespace {
int decode_shape(const InferdKvTable* t, const uint64_t* seqs, int32_t n, int32_t n_steps, int32_t* max_pages,
                 int32_t* need_pages) {
  if (!t || n <= 0 || !seqs || n_steps <= 0) return inferd_fail(INFERD_ERR_ARG, "kv decode batch: bad argument");
  int32_t mp = 1, need = 0;
  for (int32_t i = 0; i < n; ++i) {
    auto it = t->seqs.find(seqs[i]);
    if (it == t->seqs.end()) return inferd_fail(INFERD_ERR_ARG, "kv decode batch: sequence not reserved");
    for (int32_t j = 0; j < i; ++j)
      if (seqs[j] == seqs[i]) return inferd_fail(INFERD_ERR_ARG, "kv decode batch: a sequence may appear only once");
    const int32_t pg = pages_for((int64_t)it->second.length + n_steps);
    need += std::max(0, pg - (int32_t)it->second.pages.size());
    mp = std::max(mp, std::max(pg, (int32_t)it->second.pages.size()));
  }
  *max_pages = mp;
  *need_pages = need;
  return INFERD_OK;
}
}  // namespace

extern "C" int64_t inferd_kv_decode_batch_words(const InferdKvTable* t, const uint64_t* seqs, int32_t n,
                                                int32_t n_steps) {
  int32_t mp, need;
  if (decode_shape(t, seqs, n, n_steps, &mp, &need) != INFERD_OK) return -1;
  return (int64_t)n + 1 + 2 * (int64_t)n + n + (int64_t)n * mp;
}

extern "C" int inferd_kv_build_decode_batch(InferdKvTable* t, const uint64_t* seqs, int32_t n, int32_t n_steps,
                                            int32_t* host, int64_t words, const void* device_base, InferdBatch* out) {
  int32_t mp, need;
  if (int rc = decode_shape(t, seqs, n, n_steps, &mp, &need); rc != INFERD_OK) return rc;
  const int64_t want = (int64_t)n + 1 + 2 * (int64_t)n + n + (int64_t)n * mp;
  if (!host || !out || words < want) return inferd_fail(INFERD_ERR_ARG, "kv_build_decode_batch: host buffer too small");
  if (need > (int32_t)t->free.size())
    return inferd_fail(INFERD_ERR_NOMEM, "KV pool exhausted: need " + std::to_string(need) + " pages, " +
                                             std::to_string(t->free.size()) + " free of " + std::to_string(t->n_pages));
  for (int32_t i = 0; i < n; ++i)
    if (int rc = inferd_kv_reserve(t, seqs[i], n_steps); rc != INFERD_OK) return rc;  // cannot fail: checked above
  // [seq_start n+1 | positions n | slots n | ctx_lens n | block_table n x mp]
  int32_t* seq_start = host;
  int32_t* pos = seq_start + n + 1;
  int32_t* slots = pos + n;
  int32_t* ctx = slots + n;
  int32_t* table = ctx + n;
  std::fill(host, host + want, 0);
  int32_t max_len = 0;
  for (int32_t i = 0; i < n; ++i) {
    const auto& s = t->seqs.at(seqs[i]);
    seq_start[i] = i;
    ctx[i] = s.length;
    max_len = std::max(max_len, s.length);
    std::copy(s.pages.begin(), s.pages.end(), table + (int64_t)i * mp);
  }
  seq_start[n] = n;
  const int32_t* base = (const int32_t*)device_base;
  *out = InferdBatch{n, n, 1, max_len + n_steps, mp, 1, base, base + (n + 1), base + (2 * n + 1), base + (3 * n + 1),
                     base + (4 * n + 1)};
  return INFERD_OK;
}
