/* A non-Python host of the span engine's KV page table (include/inferd_span.h, "KV page
 * table"): plain C, no device calls, linked against libinferd_span.so.  It does what a
 * cgo / JNI / N-API binding of the reference's cache bookkeeping would do
 * (qwen3_server_module.py:220,253 -- a cache per session id, appended to by every call;
 * client.py:244-266 -- cache_position = past .. past + T - 1) and prints one line per check.
 * Built and run by tests/test_host.py::test_c_host_kv_table (gcc, CPU only). */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "inferd_span.h"

static int fails = 0;
#define CHECK(cond, what)                                                     \
  do {                                                                        \
    if (cond) {                                                               \
      printf("ok   %s\n", what);                                             \
    } else {                                                                  \
      printf("FAIL %s (%s)\n", what, inferd_last_error());                  \
      ++fails;                                                                \
    }                                                                         \
  } while (0)

int main(void) {
  InferdKvTable* kv = NULL;
  CHECK(inferd_kv_create(8, &kv) == INFERD_OK && kv, "create 8 pages");

  /* session 17: a 100-token prompt (prefill), then one decode token */
  const uint64_t s17 = 17, s42 = 42;
  CHECK(inferd_kv_reserve(kv, s17, 100) == INFERD_OK, "reserve 100 tokens for session 17");
  int32_t len = 0, np = 0, nfree = 0;
  inferd_kv_query(kv, s17, &len, &np);
  CHECK(len == 0 && np == 2, "session 17: 0 cached, 2 pages");

  int32_t n_new[2] = {100, 0};
  uint64_t seqs[2] = {s17, s42};
  int64_t words = inferd_kv_batch_words(kv, seqs, n_new, 1);
  CHECK(words == 1 + 1 + 2 * 100 + 1 + 2, "prefill descriptor words");
  int32_t* host = (int32_t*)malloc((size_t)words * 4);
  InferdBatch b;
  const void* dev = (const void*)0x1000; /* where the caller would copy the words */
  CHECK(inferd_kv_build_batch(kv, seqs, n_new, 1, host, words, dev, &b) == INFERD_OK, "build prefill batch");
  CHECK(b.n_seqs == 1 && b.n_tokens == 100 && b.max_q_len == 100 && b.max_ctx_len == 100 && !b.decode,
        "prefill batch shape");
  CHECK(host[0] == 0 && host[1] == 100, "seq_start");
  CHECK(host[2] == 0 && host[2 + 99] == 99, "positions 0..99");
  CHECK(host[2 + 100 + 64] == 1 * 64 + 0, "slot of token 64 = page 1, offset 0");
  CHECK((const char*)b.positions == (const char*)dev + 4 * 2, "device pointers into the caller's buffer");
  free(host);
  CHECK(inferd_kv_advance(kv, s17, 100) == INFERD_OK, "advance 100");

  /* the decode step: session 17 continues at position 100, session 42 starts */
  CHECK(inferd_kv_reserve(kv, s17, 1) == INFERD_OK && inferd_kv_reserve(kv, s42, 1) == INFERD_OK,
        "reserve one decode token each");
  n_new[0] = 1;
  n_new[1] = 1;
  words = inferd_kv_batch_words(kv, seqs, n_new, 2);
  host = (int32_t*)malloc((size_t)words * 4);
  CHECK(inferd_kv_build_batch(kv, seqs, n_new, 2, host, words, dev, &b) == INFERD_OK && b.decode == 1,
        "build decode batch");
  /* [seq_start 3 | positions 2 | slots 2 | ctx 2 | table 2 x 2] */
  CHECK(host[3] == 100 && host[4] == 0, "positions continue from the cache (100) and start at 0");
  CHECK(host[5] == 1 * 64 + 36 && host[6] == 2 * 64, "slots: session 17 page 1 offset 36, session 42 page 2");
  CHECK(host[7] == 101 && host[8] == 1, "ctx_lens");
  free(host);
  /* a decode-graph replay advances its whole batch with one call, all or nothing */
  CHECK(inferd_kv_advance_many(kv, seqs, 2, 1) == INFERD_OK, "advance_many: both sessions by one token");
  inferd_kv_query(kv, s17, &len, &np);
  CHECK(len == 101, "session 17 at 101 cached tokens");
  inferd_kv_query(kv, s42, &len, &np);
  CHECK(len == 1, "session 42 at 1 cached token");
  CHECK(inferd_kv_advance_many(kv, seqs, 2, 64) == INFERD_ERR_ARG, "advance_many past the pages is refused");
  inferd_kv_query(kv, s17, &len, &np);
  CHECK(len == 101, "nothing advanced on failure");

  /* errors: a session twice in one batch, unreserved tokens, an exhausted pool */
  seqs[1] = s17;
  CHECK(inferd_kv_batch_words(kv, seqs, n_new, 2) == -1, "a sequence twice is refused");
  n_new[0] = 65;
  seqs[0] = s42;
  CHECK(inferd_kv_batch_words(kv, seqs, n_new, 1) == -1, "tokens past the reserved pages are refused");
  inferd_kv_free_pages(kv, &nfree);
  CHECK(inferd_kv_reserve(kv, 99, 64 * (nfree + 1)) == INFERD_ERR_NOMEM, "exhausted pool: INFERD_ERR_NOMEM");
  int32_t nfree2 = 0;
  inferd_kv_free_pages(kv, &nfree2);
  CHECK(nfree2 == nfree, "nothing taken on failure");

  /* release returns the pages; a released session's first page is handed out first */
  int32_t pg[4];
  inferd_kv_pages(kv, s17, pg, 4);
  CHECK(inferd_kv_release(kv, s17) == INFERD_OK, "release session 17");
  inferd_kv_free_pages(kv, &nfree2);
  CHECK(nfree2 == nfree + 2, "its two pages are free again");
  int32_t q[1];
  inferd_kv_reserve(kv, 7, 1);
  inferd_kv_pages(kv, 7, q, 1);
  CHECK(q[0] == pg[0], "the released first page is reused first");
  inferd_kv_destroy(kv);
  printf("%s\n", fails ? "C HOST FAILED" : "C HOST OK");
  return fails ? 1 : 0;
}
