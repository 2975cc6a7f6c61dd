// ARCHIVED (round 5): this lab no longer builds against the tree -- it includes
// ../inferd_amd/csrc/attn_prefill.hip and calls launch_attn_decode_shape, both removed in round 4.
// Kept as the record of the round-3 decode-attention shape sweeps.
// Decode-attention design lab: the engine's kernel (attention.hip, included) at its default
// shape and every (waves per workgroup, chunks) shape, on B sequences x ctx tokens x KV heads
// with the paged KV pool rotated over > 1 GB (no Infinity-Cache reuse across launches, as in
// a 36-layer step).  New variants are developed here against the engine kernel.
// Standalone; not part of the engine.  Build + run on the GPU box:
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 -I inferd_amd/csrc tools/attn_lab.hip -o /tmp/attn_lab && /tmp/attn_lab
#include "../inferd_amd/csrc/attention.hip"
#include "../inferd_amd/csrc/attn_prefill.hip"

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

// Control: the decode kernel's exact read pattern (grid (nc, KV, B), each workgroup's pages,
// 32-token half-page items dealt over NW waves, 16 B per lane) with no compute -- the
// achievable rate of this access pattern.  DEPTH items in flight per wave.
template <int NW, int DEPTH>
__global__ __launch_bounds__(NW * 64) void stream_kv_kernel(const u16* __restrict__ kv, AttnBatch b, int KV, int nc,
                                                            unsigned* __restrict__ sink) {
  const int c = blockIdx.x, g = blockIdx.y, s = blockIdx.z;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int np = (b.ctx_lens[s] + KV_PAGE - 1) / KV_PAGE;
  const int p0 = c * np / nc, p1 = (c + 1) * np / nc;
  const int* bt = b.block_table + (int64_t)s * b.max_pages;
  unsigned x = 0;
  const int n_items = 2 * (p1 - p0);
  for (int u0 = wave; u0 < n_items; u0 += NW * DEPTH) {
    bf16x8 r[DEPTH][16];
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      const int u = u0 + d * NW;
      if (u >= n_items) break;
      const int phys = bt[p0 + (u >> 1)];
      const u16* kb = kv + kv_block(phys, 0, g, KV) + (u & 1) * (KV_BLOCK_ELEMS / 2);
      const u16* vb = kv + kv_block(phys, 1, g, KV) + (u & 1) * (KV_BLOCK_ELEMS / 2);
#pragma unroll
      for (int i = 0; i < 8; ++i) r[d][i] = *(const bf16x8*)(kb + i * 512 + lane * 8);
#pragma unroll
      for (int i = 0; i < 8; ++i) r[d][8 + i] = *(const bf16x8*)(vb + i * 512 + lane * 8);
    }
#pragma unroll
    for (int d = 0; d < DEPTH; ++d)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
        const u32x4_t w = __builtin_bit_cast(u32x4_t, r[d][i]);
        x ^= w[0] ^ w[1] ^ w[2] ^ w[3];
      }
  }
  if (x == 0x12345u) sink[0] = x;
}

// Control 1b: the same work split (grid (nc, KV, B), 32-token items over NW waves) but
// every workgroup's pages contiguous in memory (a head-major KV layout): what the page
// layout costs the decode read.
template <int NW, int DEPTH>
__global__ __launch_bounds__(NW * 64) void stream_contig_kernel(const u16* __restrict__ kv, int np, int nc,
                                                                unsigned* __restrict__ sink) {
  const int c = blockIdx.x, g = blockIdx.y, s = blockIdx.z;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int p0 = c * np / nc, p1 = (c + 1) * np / nc;
  // region of (s, g): np pages x (K 16 KiB + V 16 KiB), contiguous
  const u16* base = kv + ((int64_t)(s * gridDim.y + g) * np) * 2 * KV_BLOCK_ELEMS;
  unsigned x = 0;
  const int n_items = 2 * (p1 - p0);
  for (int u0 = wave; u0 < n_items; u0 += NW * DEPTH) {
    bf16x8 r[DEPTH][16];
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      const int u = u0 + d * NW;
      if (u >= n_items) break;
      const u16* kb = base + (int64_t)(p0 + (u >> 1)) * 2 * KV_BLOCK_ELEMS + (u & 1) * (KV_BLOCK_ELEMS / 2);
      const u16* vb = kb + KV_BLOCK_ELEMS;
#pragma unroll
      for (int i = 0; i < 8; ++i) r[d][i] = *(const bf16x8*)(kb + i * 512 + lane * 8);
#pragma unroll
      for (int i = 0; i < 8; ++i) r[d][8 + i] = *(const bf16x8*)(vb + i * 512 + lane * 8);
    }
#pragma unroll
    for (int d = 0; d < DEPTH; ++d)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
        const u32x4_t w = __builtin_bit_cast(u32x4_t, r[d][i]);
        x ^= w[0] ^ w[1] ^ w[2] ^ w[3];
      }
  }
  if (x == 0x12345u) sink[0] = x;
}

// Control 2: a flat read of the same number of bytes (contiguous, grid-stride, 16 B per lane,
// UNROLL loads in flight per lane) -- the floor for a one-shot ~134 MB read.
template <int UNROLL>
__global__ __launch_bounds__(256) void flat_read_kernel(const bf16x8* __restrict__ p, size_t n, unsigned* sink) {
  unsigned x = 0;
  const size_t stride = (size_t)gridDim.x * 256;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride * UNROLL) {
    bf16x8 r[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) r[u] = (i + u * stride < n) ? p[i + u * stride] : bf16x8{};
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
      const u32x4_t w = __builtin_bit_cast(u32x4_t, r[u]);
      x ^= w[0] ^ w[1] ^ w[2] ^ w[3];
    }
  }
  if (x == 0x12345u) sink[0] = x;
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 16;
  const int ctx = argc > 2 ? atoi(argv[2]) : 2100;
  const int H = 32, KV = 8;
  const int np = (ctx + 63) / 64;
  const size_t pool_elems = (size_t)((B * np + KV_SUPER - 1) / KV_SUPER * KV_SUPER) * 2 * KV * KV_BLOCK_ELEMS;
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
  unsigned* sink;
  CHECK(hipMalloc(&sink, 64));
  auto control = [&](const char* name, auto launch) {  // time only
    for (int it = 0; it < R; ++it) launch(pools[it % R]);
    const int iters = 6 * R;
    CHECK(hipEventRecord(e0));
    for (int it = 0; it < iters; ++it) launch(pools[it % R]);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / iters;
    printf("  %-26s %8.2f us  %7.0f GB/s  (read-only control)\n", name, us, bytes / (us * 1e-6) / 1e9);
  };
  // flat one-shot read floors at the decode step's per-kernel byte counts (Qwen3-8B B=16:
  // o 33.5, q/k/v 50.3, down 100.7, attention 134.2, gate/up 201.3 MB)
  for (double mb : {33.5, 50.3, 100.7, 134.2, 201.3}) {
    const size_t nv = (size_t)(mb * 1e6 / 16);
    if (nv * 16 > pool_bytes) continue;
    for (int wg : {1024, 2048, 4096}) {
      for (int it = 0; it < R; ++it)
        hipLaunchKernelGGL((flat_read_kernel<4>), dim3(wg), dim3(256), 0, 0, (const bf16x8*)pools[it % R], nv, sink);
      const int iters = 6 * R;
      CHECK(hipEventRecord(e0));
      for (int it = 0; it < iters; ++it)
        hipLaunchKernelGGL((flat_read_kernel<4>), dim3(wg), dim3(256), 0, 0, (const bf16x8*)pools[it % R], nv, sink);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      const double us = ms * 1e3 / iters;
      printf("  flat read %6.1f MB  %4d WG  %8.2f us  %7.0f GB/s\n", mb, wg, us, mb * 1e6 / (us * 1e-6) / 1e9);
    }
  }
  const size_t nvec = (size_t)(bytes / 16);
  control("flat read 1024 WG x8", [&](u16* kvp) {
    hipLaunchKernelGGL((flat_read_kernel<8>), dim3(1024), dim3(256), 0, 0, (const bf16x8*)kvp, nvec, sink);
  });
  control("flat read 2048 WG x4", [&](u16* kvp) {
    hipLaunchKernelGGL((flat_read_kernel<4>), dim3(2048), dim3(256), 0, 0, (const bf16x8*)kvp, nvec, sink);
  });
  control("flat read 4096 WG x4", [&](u16* kvp) {
    hipLaunchKernelGGL((flat_read_kernel<4>), dim3(4096), dim3(256), 0, 0, (const bf16x8*)kvp, nvec, sink);
  });
  control("contig nw8 nc2 depth2", [&](u16* kvp) {
    hipLaunchKernelGGL((stream_contig_kernel<8, 2>), dim3(2, KV, B), dim3(512), 0, 0, kvp, np, 2, sink);
  });
  control("contig nw8 nc4 depth2", [&](u16* kvp) {
    hipLaunchKernelGGL((stream_contig_kernel<8, 2>), dim3(4, KV, B), dim3(512), 0, 0, kvp, np, 4, sink);
  });
  control("stream nw8 nc2 depth2", [&](u16* kvp) {
    hipLaunchKernelGGL((stream_kv_kernel<8, 2>), dim3(2, KV, B), dim3(512), 0, 0, kvp, ab, KV, 2, sink);
  });
  control("stream nw8 nc2 depth4", [&](u16* kvp) {
    hipLaunchKernelGGL((stream_kv_kernel<8, 4>), dim3(2, KV, B), dim3(512), 0, 0, kvp, ab, KV, 2, sink);
  });
  control("stream nw8 nc4 depth2", [&](u16* kvp) {
    hipLaunchKernelGGL((stream_kv_kernel<8, 2>), dim3(4, KV, B), dim3(512), 0, 0, kvp, ab, KV, 4, sink);
  });
  control("stream nw4 nc4 depth4", [&](u16* kvp) {
    hipLaunchKernelGGL((stream_kv_kernel<4, 4>), dim3(4, KV, B), dim3(256), 0, 0, kvp, ab, KV, 4, sink);
  });
  control("stream nw8 nc1 depth2", [&](u16* kvp) {
    hipLaunchKernelGGL((stream_kv_kernel<8, 2>), dim3(1, KV, B), dim3(512), 0, 0, kvp, ab, KV, 1, sink);
  });
  control("stream nw8 nc1 depth4", [&](u16* kvp) {
    hipLaunchKernelGGL((stream_kv_kernel<8, 4>), dim3(1, KV, B), dim3(512), 0, 0, kvp, ab, KV, 1, sink);
  });
  control("stream nw16 nc1 depth4", [&](u16* kvp) {
    hipLaunchKernelGGL((stream_kv_kernel<16, 4>), dim3(1, KV, B), dim3(1024), 0, 0, kvp, ab, KV, 1, sink);
  });
  control("stream nw16 nc1 depth2", [&](u16* kvp) {
    hipLaunchKernelGGL((stream_kv_kernel<16, 2>), dim3(1, KV, B), dim3(1024), 0, 0, kvp, ab, KV, 1, sink);
  });
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
