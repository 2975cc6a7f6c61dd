/* A non-Python GPU host of the span engine: plain C over include/inferd_span.h and the HIP
 * runtime's C API (hipMalloc / hipMemcpy / streams) -- no Python, no torch.  It drives a span the
 * way a cgo / JNI / N-API binding of the reference's node would: PartitionedQwen2.forward
 * (partitioned_models.py:145-168) called token by token as send_message.py:46-60 does, with the
 * per-session KV cache of Qwen3Server.send (qwen3_server_module.py:220,237-255) kept in the
 * engine's native page table (client.py:244-266: cache_position = past .. past + T - 1).
 *
 * One span holds the whole model (embedding, layers, final norm, lm_head) with the counter-
 * generated synthetic weights; B sessions are prefilled in one call, then decoded greedily, one
 * forward call per step for all B, each feeding back its own argmax (next_ids).  The host sizes
 * nothing from headers it does not own: workspace rows and pages come from the config it passes.
 * Output, one line per session: "ids <b>: <next id after the prompt> <decode ids...>"; then "ok".
 * tests/test_gpu_span.py::test_c_host_span_greedy runs it and compares every id with the torch
 * extension's run of the same span (bit-identical kernels: the ids must match exactly).
 *
 *   usage: span_host <tiny|qwen3-0.6b> <seed> <sessions> <prompt_len> <steps>
 * Built by __graft_entry__.build() (hipcc, C only, linked against libinferd_span.so). */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "inferd_span.h"

#define HIP_OK(x)                                                                      \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                         \
    }                                                                                  \
  } while (0)
#define INF_OK(x)                                                                            \
  do {                                                                                       \
    if ((x) != INFERD_OK) {                                                                  \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, inferd_last_error());        \
      exit(3);                                                                               \
    }                                                                                        \
  } while (0)

/* the prompt token t of session b (the test builds the same ids) */
static int32_t prompt_id(int b, int t, int vocab) { return (int32_t)((7919LL * t + 104729LL * b + 17) % vocab); }

/* Build the batch of n sessions with n_new[i] new tokens each through the page table, copy its
 * words to the device buffer `dev_words` (capacity cap int32) and return the descriptor. */
static InferdBatch build(InferdKvTable* kv, const uint64_t* seqs, const int32_t* n_new, int n, int32_t* host,
                         int32_t* dev_words, int64_t cap, hipStream_t st) {
  InferdBatch b;
  const int64_t words = inferd_kv_batch_words(kv, seqs, n_new, n);
  if (words < 0 || words > cap) {
    fprintf(stderr, "batch words %lld (cap %lld): %s\n", (long long)words, (long long)cap, inferd_last_error());
    exit(4);
  }
  INF_OK(inferd_kv_build_batch(kv, seqs, n_new, n, host, words, dev_words, &b));
  HIP_OK(hipMemcpyAsync(dev_words, host, (size_t)words * 4, hipMemcpyHostToDevice, st));
  return b;
}

int main(int argc, char** argv) {
  if (argc != 6) {
    fprintf(stderr, "usage: %s <tiny|qwen3-0.6b> <seed> <sessions> <prompt_len> <steps>\n", argv[0]);
    return 1;
  }
  InferdSpanConfig c;
  memset(&c, 0, sizeof c);
  if (!strcmp(argv[1], "tiny")) { /* tests' tiny Qwen3 (inferd_amd/runtime.py MODELS) */
    c.hidden = 256, c.intermediate = 512, c.heads = 4, c.kv_heads = 2, c.vocab = 1024, c.n_layers = 4;
  } else if (!strcmp(argv[1], "qwen3-0.6b")) { /* qwen3_config.py:10-24 */
    c.hidden = 1024, c.intermediate = 3072, c.heads = 16, c.kv_heads = 8, c.vocab = 151936, c.n_layers = 28;
  } else {
    fprintf(stderr, "unknown model %s\n", argv[1]);
    return 1;
  }
  const uint64_t seed = strtoull(argv[2], NULL, 10);
  const int B = atoi(argv[3]), T = atoi(argv[4]), steps = atoi(argv[5]);
  if (B < 1 || B > 64 || T < 1 || steps < 0) {
    fprintf(stderr, "bad sizes\n");
    return 1;
  }
  const int pages_per_seq = (T + steps + INFERD_KV_PAGE_TOKENS - 1) / INFERD_KV_PAGE_TOKENS;
  c.head_dim = 128, c.first_layer = 0, c.has_embed = 1, c.has_lm_head = 1;
  c.rms_eps = 1e-6f, c.rope_theta = 1e6f, c.max_positions = 8192;
  c.kv_pages = B * pages_per_seq + 4, c.max_tokens = B * T, c.max_seqs = B;

  hipStream_t st;
  HIP_OK(hipStreamCreate(&st));
  InferdSpan* span = NULL;
  INF_OK(inferd_span_create(&c, &span));
  INF_OK(inferd_span_init_synthetic(span, seed, st));
  InferdKvTable* kv = NULL;
  INF_OK(inferd_kv_create(c.kv_pages, &kv));

  uint64_t* seqs = (uint64_t*)malloc(sizeof(uint64_t) * B);
  int32_t* n_new = (int32_t*)malloc(sizeof(int32_t) * B);
  int32_t* ids_h = (int32_t*)malloc(sizeof(int32_t) * B * T);
  int32_t* out_ids = (int32_t*)malloc(sizeof(int32_t) * B * (steps + 1));
  for (int b = 0; b < B; ++b) {
    seqs[b] = 1000 + (uint64_t)b;  /* caller-chosen session keys */
    INF_OK(inferd_kv_reserve(kv, seqs[b], T + steps));
    for (int t = 0; t < T; ++t) ids_h[b * T + t] = prompt_id(b, t, c.vocab);
  }
  /* the descriptor's worst case: the prefill call (B * T tokens) */
  for (int b = 0; b < B; ++b) n_new[b] = T;
  const int64_t cap = inferd_kv_batch_words(kv, seqs, n_new, B);
  int32_t* words_h = (int32_t*)malloc((size_t)cap * 4);
  int32_t *words_d, *ids_d, *next_d;
  HIP_OK(hipMalloc((void**)&words_d, (size_t)cap * 4));
  HIP_OK(hipMalloc((void**)&ids_d, sizeof(int32_t) * B * T));
  HIP_OK(hipMalloc((void**)&next_d, sizeof(int32_t) * B));

  /* prefill: every session's prompt in one call; next_ids = argmax of each last row */
  InferdBatch bt = build(kv, seqs, n_new, B, words_h, words_d, cap, st);
  HIP_OK(hipMemcpyAsync(ids_d, ids_h, sizeof(int32_t) * B * T, hipMemcpyHostToDevice, st));
  INF_OK(inferd_span_forward(span, &bt, ids_d, NULL, NULL, next_d, NULL, NULL, st));
  HIP_OK(hipMemcpyAsync(out_ids, next_d, sizeof(int32_t) * B, hipMemcpyDeviceToHost, st));
  HIP_OK(hipStreamSynchronize(st));
  for (int b = 0; b < B; ++b) INF_OK(inferd_kv_advance(kv, seqs[b], T));

  /* decode: one token per session per call, fed from the previous step's greedy ids */
  for (int b = 0; b < B; ++b) n_new[b] = 1;
  for (int s = 0; s < steps; ++s) {
    bt = build(kv, seqs, n_new, B, words_h, words_d, cap, st);
    HIP_OK(hipMemcpyAsync(ids_d, out_ids + s * B, sizeof(int32_t) * B, hipMemcpyHostToDevice, st));
    INF_OK(inferd_span_forward(span, &bt, ids_d, NULL, NULL, next_d, NULL, NULL, st));
    HIP_OK(hipMemcpyAsync(out_ids + (s + 1) * B, next_d, sizeof(int32_t) * B, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    INF_OK(inferd_kv_advance_many(kv, seqs, B, 1));
  }
  int32_t flags = 0;
  INF_OK(inferd_span_error_flags(span, &flags));
  if (flags) {
    fprintf(stderr, "device error flags %d\n", flags);
    return 5;
  }
  for (int b = 0; b < B; ++b) {
    printf("ids %d:", b);
    for (int s = 0; s <= steps; ++s) printf(" %d", out_ids[s * B + b]);
    printf("\n");
  }
  printf("ok\n");
  inferd_kv_destroy(kv);
  inferd_span_destroy(span);
  HIP_OK(hipFree(words_d));
  HIP_OK(hipFree(ids_d));
  HIP_OK(hipFree(next_d));
  HIP_OK(hipStreamDestroy(st));
  free(seqs), free(n_new), free(ids_h), free(out_ids), free(words_h);
  return 0;
}
