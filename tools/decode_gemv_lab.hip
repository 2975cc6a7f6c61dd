// Decode GEMV lab: times the ENGINE's decode GEMV (inferd_amd/csrc/gemm.hip, included here) per
// RMSNorm mode on the Qwen3-8B decode shapes, B = 16 rows, weights rotated over > 1 GB so no
// launch reuses the Infinity Cache (as in a 36-layer step).  DN_PROBE builds time the parts of
// the exact norm (1: no row-scale prologue, 2: no A-fragment normalisation).  GPU box:
//   for p in 0 1 2 3 4 5; do hipcc --offload-arch=gfx950 -O3 -std=c++20 -DDN_PROBE=$p \
//       tools/decode_gemv_lab.hip -o /tmp/gl$p && /tmp/gl$p; done
#include "../inferd_amd/csrc/elementwise.hip"
#include "../inferd_amd/csrc/gemm.hip"

#include <stdio.h>

#include <vector>

#define CHECK(x)                                                                \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

int main() {
  const int M = 16, h = 4096, I = 12288, qkvN = 6144;
  const int ROT = 8;
  const size_t wbytes = (size_t)2 * I * h * 2;  // the largest packed weight (gate/up)
  std::vector<u16*> W(ROT);
  for (auto& p : W) {
    CHECK(hipMalloc((void**)&p, wbytes));
    CHECK(hipMemset(p, 0x3c, wbytes));  // small bf16 values
  }
  u16 *A, *C, *R, *nw, *act;
  float *ssq, *part, *ssq_out;
  CHECK(hipMalloc((void**)&A, (size_t)M * I * 2));
  CHECK(hipMalloc((void**)&act, (size_t)M * I * 2));
  CHECK(hipMalloc((void**)&C, (size_t)M * I * 2));
  CHECK(hipMalloc((void**)&R, (size_t)M * h * 2));
  CHECK(hipMalloc((void**)&nw, (size_t)h * 2));
  CHECK(hipMalloc((void**)&ssq, (size_t)(h / 16) * 64 * 4));
  CHECK(hipMalloc((void**)&ssq_out, (size_t)(h / 16) * 64 * 4));
  CHECK(hipMalloc((void**)&part, (size_t)4 * M * qkvN * 4));
  CHECK(hipMemset(A, 0x3c, (size_t)M * I * 2));
  CHECK(hipMemset(act, 0x3c, (size_t)M * I * 2));
  CHECK(hipMemset(R, 0, (size_t)M * h * 2));
  CHECK(hipMemset(nw, 0x3f, (size_t)h * 2));
  CHECK(hipMemset(ssq, 0x3f, (size_t)(h / 16) * 64 * 4));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const RowNorm fold = {1e-6f, nullptr};
  const DecodeNorm ex = {DN_EXACT, 1e-6f, ssq, h / 16, nw};
  const DecodeNorm none = {DN_NONE, 1e-6f, nullptr, 0, nullptr};
  auto run = [&](const char* name, auto fn) {
    for (int i = 0; i < 2 * ROT; ++i) fn(W[i % ROT]);
    CHECK(hipDeviceSynchronize());
    const int n = 20 * ROT;
    CHECK(hipEventRecord(e0));
    for (int i = 0; i < n; ++i) fn(W[i % ROT]);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    printf("DN_PROBE=%d %-28s %8.2f us\n", DN_PROBE, name, ms * 1e3f / n);
  };
  run("gateup none", [&](u16* w) { launch_gemm(A, h, w, M, I, h, C, I, nullptr, 0, EPI_SILU, nullptr, 0, nullptr, nullptr, &none); });
  run("gateup fold", [&](u16* w) { launch_gemm(A, h, w, M, I, h, C, I, nullptr, 0, EPI_SILU, nullptr, 0, &fold); });
  run("gateup exact", [&](u16* w) { launch_gemm(A, h, w, M, I, h, C, I, nullptr, 0, EPI_SILU, nullptr, 0, nullptr, nullptr, &ex); });
  const DecodeNorm pf = {DN_FOLD, 1e-6f, nullptr, 0, nullptr};
  run("qkv split2 none", [&](u16* w) { launch_gemm_decode_partial(A, h, w, M, qkvN, h, 2, part, nullptr, none, 0); });
  run("qkv split2 fold", [&](u16* w) { launch_gemm_decode_partial(A, h, w, M, qkvN, h, 2, part, part + 3 * M * qkvN, pf, 0); });
  run("qkv split2 exact", [&](u16* w) { launch_gemm_decode_partial(A, h, w, M, qkvN, h, 2, part, nullptr, ex, 0); });
  run("o resid", [&](u16* w) { launch_gemm(A, h, w, M, h, h, C, h, R, h, EPI_RESID, nullptr, 0); });
  run("o resid + ssq_out", [&](u16* w) { launch_gemm(A, h, w, M, h, h, C, h, R, h, EPI_RESID, nullptr, 0, nullptr, nullptr, nullptr, ssq_out); });
  run("down resid", [&](u16* w) { launch_gemm(act, I, w, M, h, I, C, h, R, h, EPI_RESID, nullptr, 0); });
  {
    static unsigned long long* keys = nullptr;
    const int V = 151936;
    if (!keys) CHECK(hipMalloc((void**)&keys, (size_t)M * (V / 16) * 8));
    // lm_head shape (V x h = 1.24 GB > the rotation buffers: one buffer pair, Infinity Cache
    // defeated by its size)
    static u16* lm = nullptr;
    if (!lm) {
      CHECK(hipMalloc((void**)&lm, (size_t)V * h * 2));
      CHECK(hipMemset(lm, 0x3c, (size_t)V * h * 2));
    }
    run("lm_head argmax", [&](u16*) { launch_gemm(A, h, lm, M, V, h, nullptr, 0, nullptr, 0, EPI_ARGMAX, keys, 0); });
    // ring shapes for the many-round lm_head grid (the launcher's DecodeCfg is tuned on the
    // one-round layer GEMVs)
    DecodeArgs a = {};
    a.M = M;
    a.A = A;
    a.lda = h;
    a.Wp = lm;
    a.KT = h / 32;
    a.n_tiles = V / 16;
    a.keys = keys;
    auto cfg = [&](const char* name, auto kern, int threads) {
      run(name, [&](u16*) { hipLaunchKernelGGL(kern, dim3(a.n_tiles), dim3(threads), 0, 0, a); });
    };
    cfg("lm_head NW8 TW4 D3", gemm_decode_kernel<1, 1, 8, 4, 3, EPI_ARGMAX, DN_NONE>, 512);
    cfg("lm_head NW8 TW4 D2", gemm_decode_kernel<1, 1, 8, 4, 2, EPI_ARGMAX, DN_NONE>, 512);
    cfg("lm_head NW8 TW2 D4", gemm_decode_kernel<1, 1, 8, 2, 4, EPI_ARGMAX, DN_NONE>, 512);
    cfg("lm_head NW4 TW4 D3", gemm_decode_kernel<1, 1, 4, 4, 3, EPI_ARGMAX, DN_NONE>, 256);
    cfg("lm_head NW4 TW4 D4", gemm_decode_kernel<1, 1, 4, 4, 4, EPI_ARGMAX, DN_NONE>, 256);
    cfg("lm_head NW4 TW8 D2", gemm_decode_kernel<1, 1, 4, 8, 2, EPI_ARGMAX, DN_NONE>, 256);
    cfg("lm_head NW16 TW2 D2", gemm_decode_kernel<1, 1, 16, 2, 2, EPI_ARGMAX, DN_NONE>, 1024);
    cfg("lm_head NW16 TW4 D2", gemm_decode_kernel<1, 1, 16, 4, 2, EPI_ARGMAX, DN_NONE>, 1024);
  }
  {
    // ring depth for the one-round o GEMV: D = 5 puts all four batches of a wave in flight
    // in the prologue (no refill in the loop at all)
    DecodeArgs a = {};
    a.M = M;
    a.A = A;
    a.lda = h;
    a.KT = h / 32;
    a.n_tiles = h / 16;
    a.C = C;
    a.ldc = h;
    a.R = R;
    a.ldr = h;
    a.ssq_out = ssq_out;
    auto cfg = [&](const char* name, auto kern) {
      run(name, [&](u16* w) {
        a.Wp = w;
        hipLaunchKernelGGL(kern, dim3(a.n_tiles), dim3(512), 0, 0, a);
      });
    };
    cfg("o NW8 TW4 D3", gemm_decode_kernel<1, 1, 8, 4, 3, EPI_RESID, DN_NONE>);
    cfg("o NW8 TW4 D4", gemm_decode_kernel<1, 1, 8, 4, 4, EPI_RESID, DN_NONE>);
    cfg("o NW8 TW4 D5", gemm_decode_kernel<1, 1, 8, 4, 5, EPI_RESID, DN_NONE>);
    cfg("o NW8 TW2 D5", gemm_decode_kernel<1, 1, 8, 2, 5, EPI_RESID, DN_NONE>);
    cfg("o NW8 TW2 D9", gemm_decode_kernel<1, 1, 8, 2, 9, EPI_RESID, DN_NONE>);
    a.A = act;
    a.lda = I;
    a.KT = I / 32;
    cfg("down NW8 TW4 D3", gemm_decode_kernel<1, 1, 8, 4, 3, EPI_RESID, DN_NONE>);
    cfg("down NW8 TW4 D4", gemm_decode_kernel<1, 1, 8, 4, 4, EPI_RESID, DN_NONE>);
    cfg("down NW8 TW4 D5", gemm_decode_kernel<1, 1, 8, 4, 5, EPI_RESID, DN_NONE>);
  }
  {
    // ring shapes for the split-K q/k/v GEMV with the exact norm (768 workgroups, 2 slices)
    DecodeArgs a = {};
    a.A = A;
    a.lda = h;
    a.KT = h / 32;
    a.n_tiles = qkvN / 16;
    a.M = M;
    a.eps = 1e-6f;
    a.part = part;
    a.ldp = qkvN;
    a.ssq_in = ssq;
    a.n_parts = h / 16;
    a.norm_w = nw;
    auto cfg = [&](const char* name, auto kern, int nwv, int ksl) {
      run(name, [&](u16* w) {
        a.Wp = w;
        hipLaunchKernelGGL(kern, dim3(a.n_tiles, ksl), dim3((nwv + 1) * 64), (dn_lds_bytes<DN_EXACT, 1>(a.KT / ksl)), 0, a);
      });
    };
    cfg("qkv x2 NW4 TW4 D3", gemm_decode_kernel<1, 1, 4, 4, 3, EPI_PARTIAL, DN_EXACT>, 4, 2);
    cfg("qkv x2 NW4 TW4 D2", gemm_decode_kernel<1, 1, 4, 4, 2, EPI_PARTIAL, DN_EXACT>, 4, 2);
    cfg("qkv x2 NW4 TW4 D4", gemm_decode_kernel<1, 1, 4, 4, 4, EPI_PARTIAL, DN_EXACT>, 4, 2);
    cfg("qkv x2 NW4 TW2 D4", gemm_decode_kernel<1, 1, 4, 2, 4, EPI_PARTIAL, DN_EXACT>, 4, 2);
    cfg("qkv x2 NW4 TW2 D6", gemm_decode_kernel<1, 1, 4, 2, 6, EPI_PARTIAL, DN_EXACT>, 4, 2);
    cfg("qkv x2 NW8 TW2 D2", gemm_decode_kernel<1, 1, 8, 2, 2, EPI_PARTIAL, DN_EXACT>, 8, 2);
    cfg("qkv x2 NW8 TW2 D4", gemm_decode_kernel<1, 1, 8, 2, 4, EPI_PARTIAL, DN_EXACT>, 8, 2);
    cfg("qkv x2 NW8 TW4 D2", gemm_decode_kernel<1, 1, 8, 4, 2, EPI_PARTIAL, DN_EXACT>, 8, 2);
    cfg("qkv x2 NW2 TW4 D4", gemm_decode_kernel<1, 1, 2, 4, 4, EPI_PARTIAL, DN_EXACT>, 2, 2);
    cfg("qkv x1 NW8 TW4 D3", gemm_decode_kernel<1, 1, 8, 4, 3, EPI_PARTIAL, DN_EXACT>, 8, 1);
    cfg("qkv x1 NW8 TW4 D4", gemm_decode_kernel<1, 1, 8, 4, 4, EPI_PARTIAL, DN_EXACT>, 8, 1);
    cfg("qkv x4 NW4 TW4 D2", gemm_decode_kernel<1, 1, 4, 4, 2, EPI_PARTIAL, DN_EXACT>, 4, 4);
    cfg("qkv x4 NW2 TW4 D4", gemm_decode_kernel<1, 1, 2, 4, 4, EPI_PARTIAL, DN_EXACT>, 2, 4);
  }
  // fragment-packed activations / residual stream (the span's decode layout)
  run("gateup exact packed", [&](u16* w) { launch_gemm(A, h, w, M, I, h, C, I, nullptr, 0, EPI_SILU, nullptr, 0, nullptr, nullptr, &ex, nullptr, GEMM_PACK_A | GEMM_PACK_C); });
  run("qkv split2 exact packed", [&](u16* w) { launch_gemm_decode_partial(A, h, w, M, qkvN, h, 2, part, nullptr, ex, 0, GEMM_PACK_A); });
  run("o resid + ssq_out packed", [&](u16* w) { launch_gemm(A, h, w, M, h, h, C, h, R, h, EPI_RESID, nullptr, 0, nullptr, nullptr, nullptr, ssq_out, GEMM_PACK_A | GEMM_PACK_R | GEMM_PACK_C); });
  run("down resid + ssq_out packed", [&](u16* w) { launch_gemm(act, I, w, M, h, I, C, h, R, h, EPI_RESID, nullptr, 0, nullptr, nullptr, nullptr, ssq_out, GEMM_PACK_A | GEMM_PACK_R | GEMM_PACK_C); });
  run("down resid + ssq_out", [&](u16* w) { launch_gemm(act, I, w, M, h, I, C, h, R, h, EPI_RESID, nullptr, 0, nullptr, nullptr, nullptr, ssq_out); });
  return 0;
}
