// Decode-attention design lab: the engine's kernel (attention.hip, included) at its default
// shape and every (waves per workgroup, chunks) shape, on B sequences x ctx tokens x KV heads
// with the paged KV pool rotated over > 1 GB (no Infinity-Cache reuse across launches, as in
// a 36-layer step).  New variants are developed here against the engine kernel.
// Standalone; not part of the engine.  Build + run on the GPU box:
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 -I inferd_amd/csrc tools/attn_lab.hip -o /tmp/attn_lab && /tmp/attn_lab
#include "../inferd_amd/csrc/attention.hip"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

__global__ void fill_kernel(u16* p, size_t n, uint64_t seed) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint64_t r = splitmix64(seed ^ i);
    float f = ((float)(r & 0xFFFF) / 65536.0f - 0.5f) * 2.0f;
    p[i] = f2bf(f);
  }
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 16;
  const int ctx = argc > 2 ? atoi(argv[2]) : 2100;
  const int H = 32, KV = 8;
  const int np = (ctx + 63) / 64;
  const size_t pool_elems = (size_t)B * np * 2 * KV * KV_BLOCK_ELEMS;
  const size_t pool_bytes = pool_elems * 2;
  const int R = (int)((1536ull << 20) / pool_bytes) + 1;
  std::vector<u16*> pools(R);
  for (int r = 0; r < R; ++r) {
    CHECK(hipMalloc(&pools[r], pool_bytes));
    hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, pools[r], pool_elems, 11ull + r);
  }
  // batch: sequence b owns pages [b*np, (b+1)*np), last token at position ctx-1
  std::vector<int> h_start(B + 1), h_pos(B), h_ctx(B), h_bt((size_t)B * np);
  for (int i = 0; i <= B; ++i) h_start[i] = i;
  for (int i = 0; i < B; ++i) {
    h_pos[i] = ctx - 1;
    h_ctx[i] = ctx;
    for (int p = 0; p < np; ++p) h_bt[(size_t)i * np + p] = i * np + p;
  }
  int *d_start, *d_pos, *d_ctx, *d_bt;
  CHECK(hipMalloc(&d_start, (B + 1) * 4));
  CHECK(hipMalloc(&d_pos, B * 4));
  CHECK(hipMalloc(&d_ctx, B * 4));
  CHECK(hipMalloc(&d_bt, (size_t)B * np * 4));
  CHECK(hipMemcpy(d_start, h_start.data(), (B + 1) * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_pos, h_pos.data(), B * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_ctx, h_ctx.data(), B * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_bt, h_bt.data(), (size_t)B * np * 4, hipMemcpyHostToDevice));
  AttnBatch ab;
  ab.seq_start = d_start;
  ab.positions = d_pos;
  ab.ctx_lens = d_ctx;
  ab.block_table = d_bt;
  ab.max_pages = np;
  ab.B = B;
  ab.M = B;
  ab.max_q_len = 1;
  ab.max_ctx = ctx;
  u16 *q, *out, *ref;
  CHECK(hipMalloc(&q, (size_t)B * H * 128 * 2));
  CHECK(hipMalloc(&out, (size_t)B * H * 128 * 2));
  CHECK(hipMalloc(&ref, (size_t)B * H * 128 * 2));
  hipLaunchKernelGGL(fill_kernel, dim3(256), dim3(256), 0, 0, q, (size_t)B * H * 128, 5ull);
  const size_t wsb = attn_decode_ws_bytes(B, H, ctx);
  float* ws;
  CHECK(hipMalloc(&ws, wsb));
  CHECK(hipMemset(ws, 0, wsb));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const double bytes = (double)B * ctx * KV * 128 * 2 * 2;
  printf("B=%d ctx=%d H=%d KV=%d: %.1f MB KV per launch, %d pools rotated\n", B, ctx, H, KV, bytes / 1e6, R);
  // reference output: engine kernel, default ppw
  launch_attn_decode(q, pools[0], ab, H, KV, 1.0f / sqrtf(128.f), ref, ws, 0);
  CHECK(hipDeviceSynchronize());
  std::vector<u16> hr((size_t)B * H * 128), ho((size_t)B * H * 128);
  CHECK(hipMemcpy(hr.data(), ref, hr.size() * 2, hipMemcpyDeviceToHost));
  auto bf = [](u16 v) {
    uint32_t u = (uint32_t)v << 16;
    float f;
    memcpy(&f, &u, 4);
    return f;
  };
  auto run = [&](const char* name, auto launch) {
    launch(pools[0]);
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemcpy(ho.data(), out, ho.size() * 2, hipMemcpyDeviceToHost));
    double md = 0;
    for (size_t i = 0; i < ho.size(); ++i) md = fmax(md, fabs(bf(ho[i]) - bf(hr[i])));
    for (int it = 0; it < R; ++it) launch(pools[it % R]);
    const int iters = 6 * R;
    CHECK(hipEventRecord(e0));
    for (int it = 0; it < iters; ++it) launch(pools[it % R]);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / iters;
    printf("  %-26s %8.2f us  %7.0f GB/s  maxdiff %.3e\n", name, us, bytes / (us * 1e-6) / 1e9, md);
  };
  run("engine default shape", [&](u16* kvp) {
    launch_attn_decode(q, kvp, ab, H, KV, 1.0f / sqrtf(128.f), out, ws, 0);
  });
  for (int nc : {1, 2, 4, 8, 16, 32}) {
    if (nc > np) continue;
    for (int nw : {4, 8}) {
      char nm[64];
      snprintf(nm, sizeof nm, "nw%d nc=%d", nw, nc);
      run(nm, [&](u16* kvp) {
        launch_attn_decode_shape(q, kvp, ab, H, KV, 1.0f / sqrtf(128.f), out, ws, 0, nw, nc);
      });
    }
  }
  return 0;
}
