"""Per-kernel parity of the HIP path (through the C-ABI) against the CPU oracle.

Tolerances: integer/layout ops bit-exact; elementwise bf16 ops reproduce the
reference's rounding points and must match the oracle bit-for-bit on all but a
vanishing fraction of elements (1 bf16 ulp allowed where transcendental / reduction
order differs); GEMM / attention compare to an fp32 reference of the same bf16
inputs with a relative tolerance stated per test.
"""
import numpy as np
import pytest
import torch

from oracle import qwen3_ref as R
from oracle import weightgen as wg

pytestmark = pytest.mark.gpu

SEED = 1234
DEV = "cuda"


@pytest.fixture(scope="module")
def lib():
    from inferd_amd import _lib
    return _lib


def bf16_ulp_diff(a, b):
    """max difference in bf16 ulps (monotone int16 ordering)."""
    ai = a.view(torch.int16).to(torch.int32)
    bi = b.view(torch.int16).to(torch.int32)
    ai = torch.where(ai < 0, -32768 - ai, ai)
    bi = torch.where(bi < 0, -32768 - bi, bi)
    return (ai - bi).abs()


def test_weightgen_bit_exact(lib):
    for tid, name, n in ((7, "q_proj", 100003), (0xFFFF0001, "norm", 4096), (3 * 16 + 4, "q_norm", 128)):
        scale, center = wg.tensor_spec(name)
        out = torch.empty(n, dtype=torch.bfloat16, device=DEV)
        lib.check(lib.load().inferd_weightgen(out.data_ptr(), n, SEED, tid, scale, center, lib.stream_ptr()))
        ref = wg.bf16_rne_bits(wg.uniform_fp32(SEED, tid, n, scale, center))
        got = out.cpu().view(torch.int16).numpy().view(np.uint16)
        assert np.array_equal(got, ref), name


def test_pack_unpack_roundtrip(lib):
    L = lib.load()
    for N, K in ((16, 32), (48, 96), (4096, 1024)):
        w = torch.randn(N, K, device=DEV).to(torch.bfloat16)
        p = torch.empty_like(w)
        u = torch.empty_like(w)
        lib.check(L.inferd_pack_weight(w.data_ptr(), N, K, p.data_ptr(), lib.stream_ptr()))
        lib.check(L.inferd_unpack_weight(p.data_ptr(), N, K, u.data_ptr(), lib.stream_ptr()))
        assert torch.equal(w, u)
        # spot-check the documented fragment layout: tile (nt,kt), lane l, elem j
        pc, wc = p.cpu().view(-1), w.cpu()
        KT = K // 32
        for nt, kt, l, j in ((0, 0, 0, 0), (0, 0, 17, 3), (N // 16 - 1, KT - 1, 63, 7)):
            assert pc[(nt * KT + kt) * 512 + l * 8 + j] == wc[16 * nt + (l & 15), 32 * kt + 8 * (l >> 4) + j]


def test_rmsnorm_matches_oracle(lib):
    L = lib.load()
    d = R.CONFIGS["qwen3-8b"]
    for rows, cols, scale in ((16, 4096, 1.0), (7, 1024, 30.0), (3, 5120, 0.01), (2, 256, 5.0)):
        x = (torch.randn(rows, cols) * scale).to(torch.bfloat16)
        w = (1 + 0.1 * torch.randn(cols)).to(torch.bfloat16)
        ref = R.rms_norm(x, w, d.eps)
        y = torch.empty(rows, cols, dtype=torch.bfloat16, device=DEV)
        xd, wd = x.to(DEV), w.to(DEV)
        lib.check(L.inferd_rmsnorm(xd.data_ptr(), wd.data_ptr(), y.data_ptr(), rows, cols, d.eps,
                                   lib.stream_ptr()))
        ulp = bf16_ulp_diff(y.cpu(), ref)
        assert ulp.max() <= 1 and (ulp > 0).float().mean() < 2e-3, (rows, cols, ulp.max(), (ulp > 0).float().mean())


def test_rmsnorm_golden(lib):
    from golden_io import load, tensor
    u = load("units.npz")
    L = lib.load()
    d = R.CONFIGS["qwen3-0.6b"]
    x = tensor(u["rms_bf16_x"])
    w = R.gen_layer_weights(d, SEED, 0)["input_layernorm"]
    y = torch.empty_like(x, device=DEV)
    xd, wd = x.to(DEV), w.to(DEV)
    lib.check(L.inferd_rmsnorm(xd.data_ptr(), wd.data_ptr(), y.data_ptr(), x.shape[0], x.shape[1],
                               d.eps, lib.stream_ptr()))
    ulp = bf16_ulp_diff(y.cpu(), tensor(u["rms_bf16_y"]))
    assert ulp.max() <= 1 and (ulp > 0).float().mean() < 2e-3


def _gemm(lib, a, w, epi, r=None):
    L = lib.load()
    N, K = w.shape
    n_out = N // 2 if epi == lib.EPI_SILU else N
    wp = torch.empty_like(w)
    lib.check(L.inferd_pack_weight(w.data_ptr(), N, K, wp.data_ptr(), lib.stream_ptr()))
    c = torch.empty(a.shape[0], n_out, dtype=torch.bfloat16, device=DEV)
    lib.check(L.inferd_gemm(a.data_ptr(), wp.data_ptr(), c.data_ptr(), None if r is None else r.data_ptr(),
                            a.shape[0], n_out, K, epi, lib.stream_ptr()))
    return c


@pytest.mark.parametrize("M", [1, 5, 16, 33, 64, 65, 200, 1000])
@pytest.mark.parametrize("N,K", [(256, 256), (1024, 4096), (384, 1024)])
def test_gemm_plain_and_resid(lib, M, N, K):
    torch.manual_seed(M * 7 + N)
    a = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) * 0.03).to(torch.bfloat16)
    ref = a.float() @ w.float().t()
    c = _gemm(lib, a, w, lib.EPI_NONE)
    err = (c.float() - ref).abs().max().item()
    assert err <= 1e-2 * ref.abs().max().item() + 1e-3, err
    # bf16 rounding of an fp32 accumulator: within 1 ulp of the rounded fp32 reference
    assert (bf16_ulp_diff(c.cpu(), ref.to(torch.bfloat16).cpu()) > 1).float().mean() < 1e-3
    r = torch.randn(M, N, device=DEV).to(torch.bfloat16)
    c2 = _gemm(lib, a, w, lib.EPI_RESID, r)
    ref2 = (ref.to(torch.bfloat16).float() + r.float()).to(torch.bfloat16)
    assert (bf16_ulp_diff(c2.cpu(), ref2.cpu()) > 1).float().mean() < 1e-3


@pytest.mark.parametrize("M,K", [(1, 1024), (16, 1024), (64, 1024), (300, 1024), (16, 4096), (40, 4096),
                                 (600, 1024)])
def test_gemm_swiglu(lib, M, K):
    """Also covers the decode GEMM's split-K reduction (K = 4096 -> 4 slices at M <= 16)."""
    torch.manual_seed(M)
    I = 512
    a = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    g = (torch.randn(I, K, device=DEV) * 0.03).to(torch.bfloat16)
    u = (torch.randn(I, K, device=DEV) * 0.03).to(torch.bfloat16)
    c = _gemm(lib, a, torch.cat([g, u], 0).contiguous(), lib.EPI_SILU)
    # reference rounding points: F.silu(gate(x)) * up(x) in bf16
    gr = (a.float() @ g.float().t()).to(torch.bfloat16)
    ur = (a.float() @ u.float().t()).to(torch.bfloat16)
    ref = torch.nn.functional.silu(gr) * ur
    assert (bf16_ulp_diff(c.cpu(), ref.cpu()) > 2).float().mean() < 2e-3


@pytest.mark.parametrize("M,N,K", [(512, 512, 192), (777, 768, 1088), (2048, 1024, 4096), (1300, 256, 640),
                                   (4096, 2048, 1024), (8092, 4096, 448), (300, 384, 1024), (16500, 1024, 256),
                                   (20000, 2048, 512)])
def test_gemm_prefill_bodies(lib, M, N, K):
    """The prefill GEMM bodies on ragged M, short and long K, all epilogues: persistent
    gemm_w4p; gemm_w4 with the tail split ((2048, 1024, 4096) and (4096, 2048, 1024) cut K
    8 / 2 ways); (8092, 4096, 448): 512 whole tiles, so w4p walks two tiles per workgroup
    (ragged last row block, cross-tile prefetch, exact-count epilogue waits); (300, 384,
    1024): the 128x128 gemm_tiled; (16500, 1024, 256) and (20000, 2048, 512): >= 64 row blocks
    (ragged), so tile_order_v's row groups are 4 blocks deep."""
    torch.manual_seed(M + N + K)
    a = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) * 0.03).to(torch.bfloat16)
    ref = a.float() @ w.float().t()
    c = _gemm(lib, a, w, lib.EPI_NONE)
    assert (bf16_ulp_diff(c.cpu(), ref.to(torch.bfloat16).cpu()) > 1).float().mean() < 1e-3
    r = torch.randn(M, N, device=DEV).to(torch.bfloat16)
    c2 = _gemm(lib, a, w, lib.EPI_RESID, r)
    ref2 = (ref.to(torch.bfloat16).float() + r.float()).to(torch.bfloat16)
    assert (bf16_ulp_diff(c2.cpu(), ref2.cpu()) > 1).float().mean() < 1e-3
    half = N // 2
    c3 = _gemm(lib, a, w, lib.EPI_SILU)
    gr = ref[:, :half].to(torch.bfloat16)
    ur = ref[:, half:].to(torch.bfloat16)
    ref3 = torch.nn.functional.silu(gr) * ur
    assert (bf16_ulp_diff(c3.cpu(), ref3.cpu()) > 2).float().mean() < 2e-3


def test_qk_norm_rope_golden_and_cache(lib):
    """QK-norm + RoPE vs the reference's own output (units.npz), K/V written to the cache."""
    from golden_io import load, tensor
    from kv_layout import read_kv
    L = lib.load()
    u = load("units.npz")
    d = R.CONFIGS["qwen3-0.6b"]
    W = R.gen_layer_weights(d, SEED, 3)
    q, k = tensor(u["qkr_q"]), tensor(u["qkr_k"])  # (1,T,H,d), (1,T,KV,d)
    T = q.shape[1]
    v = torch.randn(1, T, d.kv_heads, 128).to(torch.bfloat16)
    qkv = torch.cat([q.reshape(T, -1), k.reshape(T, -1), v.reshape(T, -1)], 1).contiguous().to(DEV)
    pos = torch.from_numpy(u["qkr_pos"]).reshape(-1).to(torch.int32).to(DEV)
    cos_t = torch.empty(40960, 64, dtype=torch.bfloat16, device=DEV)
    sin_t = torch.empty_like(cos_t)
    lib.check(L.inferd_rope_table(d.rope_theta, 128, 40960, cos_t.data_ptr(), sin_t.data_ptr(), lib.stream_ptr()))
    pages = [3, 1, 5]
    slots = torch.tensor([pages[(100 + i) // 64] * 64 + (100 + i) % 64 for i in range(T)], dtype=torch.int32, device=DEV)
    from kv_layout import pool_elems
    kv = torch.zeros(pool_elems(8, d.kv_heads), dtype=torch.bfloat16, device=DEV)
    q_out = torch.empty(T, d.heads, 128, dtype=torch.bfloat16, device=DEV)
    qn_d, kn_d = W["q_norm"].to(DEV), W["k_norm"].to(DEV)
    lib.check(L.inferd_qk_norm_rope_kv(qkv.data_ptr(), pos.data_ptr(), slots.data_ptr(), qn_d.data_ptr(),
                                       kn_d.data_ptr(), cos_t.data_ptr(), sin_t.data_ptr(),
                                       q_out.data_ptr(), kv.data_ptr(), T, d.heads, d.kv_heads, d.eps,
                                       lib.stream_ptr()))
    qe = tensor(u["qkr_q_out"])[0].transpose(0, 1)  # (T,H,d)
    ke = tensor(u["qkr_k_out"])[0]                  # (KV,T,d)
    ulp = bf16_ulp_diff(q_out.cpu(), qe)
    assert ulp.max() <= 1 and (ulp > 0).float().mean() < 5e-3
    K, V = read_kv(kv, d.kv_heads, pages, 100 + T)
    ulp = bf16_ulp_diff(K[:, 100:], ke)
    assert ulp.max() <= 1 and (ulp > 0).float().mean() < 5e-3
    assert torch.equal(V[:, 100:], v[0].transpose(0, 1))


def test_rope_table_matches_hf(lib):
    from golden_io import load, tensor
    L = lib.load()
    u = load("units.npz")
    d = R.CONFIGS["qwen3-0.6b"]
    cos_t = torch.empty(40960, 64, dtype=torch.bfloat16, device=DEV)
    sin_t = torch.empty_like(cos_t)
    lib.check(L.inferd_rope_table(d.rope_theta, 128, 40960, cos_t.data_ptr(), sin_t.data_ptr(), lib.stream_ptr()))
    pos = torch.from_numpy(u["rope_pos"]).reshape(-1).long()
    c_ref = tensor(u["rope_bf16_cos"])[0][:, :64]
    s_ref = tensor(u["rope_bf16_sin"])[0][:, :64]
    assert bf16_ulp_diff(cos_t.cpu()[pos], c_ref).max() <= 1
    assert bf16_ulp_diff(sin_t.cpu()[pos], s_ref).max() <= 1
    # dense check against the oracle table for the first 4096 positions
    c, s = R.rope_cos_sin(d, torch.arange(4096)[None], torch.bfloat16)
    ulp_c = bf16_ulp_diff(cos_t.cpu()[:4096], c[0, :, :64])
    ulp_s = bf16_ulp_diff(sin_t.cpu()[:4096], s[0, :, :64])
    assert ulp_c.max() <= 1 and (ulp_c > 0).float().mean() < 1e-3
    assert ulp_s.max() <= 1 and (ulp_s > 0).float().mean() < 1e-3


def _attn_case(lib, H, KV, q_lens, past_lens, seed=0, n_pages=256):
    """Random bf16 q/K/V; K/V written into shuffled pages; compare with fp32 SDPA."""
    from inferd_amd.runtime import KvTable, SeqView
    from kv_layout import K_IDX, V_IDX, block, pool_elems
    torch.manual_seed(seed)
    L = lib.load()
    table = KvTable(n_pages)
    # scatter the free list: one-page sequences released in a random order
    for i in range(n_pages):
        table.reserve(10_000 + i, 1)
    for i in np.random.default_rng(seed).permutation(n_pages):
        table.release(10_000 + int(i))
    kv = torch.zeros(pool_elems(n_pages, KV), dtype=torch.bfloat16)
    seqs, Ks, Vs, Qs = [], [], [], []
    for j, (T, P) in enumerate(zip(q_lens, past_lens)):
        st = SeqView(table, j)
        n = T + P
        table.reserve(j, n)
        table.advance(j, P)
        K = (torch.randn(KV, n, 128) * 1.0).to(torch.bfloat16)
        V = torch.randn(KV, n, 128).to(torch.bfloat16)
        for pi, p in enumerate(st.pages):
            kk = torch.zeros(KV, 64, 128, dtype=torch.bfloat16)
            vv = torch.zeros(KV, 64, 128, dtype=torch.bfloat16)
            m = min(64, n - pi * 64)
            kk[:, :m] = K[:, pi * 64: pi * 64 + m]
            vv[:, :m] = V[:, pi * 64: pi * 64 + m]
            block(kv, KV, p, 0)[:, K_IDX.reshape(-1)] = kk.reshape(KV, -1)
            block(kv, KV, p, 1)[:, V_IDX.reshape(-1)] = vv.reshape(KV, -1)
        seqs.append((st, T))
        Ks.append(K)
        Vs.append(V)
        Qs.append((torch.randn(T, H, 128) * 1.5).to(torch.bfloat16))
    bd = table.build_batch([(st.seq, T) for st, T in seqs], DEV)
    batch = lib.batch_struct(bd.words, bd.shape)
    q = torch.cat(Qs, 0).contiguous().to(DEV)
    out = torch.empty(q.shape[0], H * 128, dtype=torch.bfloat16, device=DEV)
    ws_bytes = L.inferd_attention_workspace_bytes(len(seqs), H, max(t + p for t, p in zip(q_lens, past_lens)))
    ws = torch.zeros(max(ws_bytes, 256), dtype=torch.uint8, device=DEV)
    kv_d = kv.to(DEV)
    lib.check(L.inferd_attention(q.data_ptr(), kv_d.data_ptr(), batch, H, KV, out.data_ptr(), ws.data_ptr(),
                                 ws_bytes, lib.stream_ptr()))
    torch.cuda.synchronize()
    refs = []
    for Q, K, V, (st, T) in zip(Qs, Ks, Vs, seqs):
        o = R.attention(Q.float().transpose(0, 1)[None], K.float()[None], V.float()[None], st.length,
                        128 ** -0.5, "sdpa")
        refs.append(o[0].reshape(T, H * 128))
    ref = torch.cat(refs, 0)
    err = (out.cpu().float() - ref).abs()
    return err, ref


# Attention error bounds against fp32 SDPA (the kernels' inputs are bf16, their output is
# rounded to bf16 -- alone a relative rms error of ~1.1e-3 -- and P enters the P.V MFMA as
# bf16; prefill also rounds q * scale * log2 e to bf16, attention.hip): every element within
# ATTN_MAX_REL * max(1, max|ref|), and the rms error within ATTN_RMS_REL * rms(ref), which a
# systematic error (e.g. a wrong lazy rescale) spread over many elements cannot hide under.
ATTN_MAX_REL = 2e-2
ATTN_RMS_REL = 3e-3


def _attn_check(err, ref, name):
    rms_rel = (err.pow(2).mean().sqrt() / ref.pow(2).mean().sqrt()).item()
    mx = err.max().item()
    print(f"{name}: max|d| {mx:.3e} (max|ref| {ref.abs().max().item():.2f}), rms(d)/rms(ref) {rms_rel:.2e}")
    from parity_log import record
    record(f"attention_{name}", max_abs=mx, rms_rel=rms_rel, rms_bound=ATTN_RMS_REL)
    assert mx < ATTN_MAX_REL * max(1.0, ref.abs().max().item()), mx
    assert rms_rel <= ATTN_RMS_REL, rms_rel


@pytest.mark.parametrize("H,KV", [(32, 8), (16, 8), (64, 8), (4, 2)])
def test_attention_decode(lib, H, KV):
    err, ref = _attn_case(lib, H, KV, [1] * 5, [0, 63, 64, 700, 2100], seed=H)
    _attn_check(err, ref, f"decode_H{H}_KV{KV}")


@pytest.mark.parametrize("q_lens,past", [([1], [5999]), ([1, 1], [5999, 3000])], ids=["b1_ctx6000", "b2_ctx6000_3001"])
def test_attention_decode_many_chunks(lib, q_lens, past):
    """Few sequences at long context split into many chunks per (sequence, kv head): 23 chunks for
    one sequence at 6000 tokens, 16 for two -- the last-arriving chunk merges them 8 at a time
    (attention.hip), so these exercise several merge blocks and a partial last block."""
    err, ref = _attn_case(lib, 32, 8, q_lens, past, seed=7)
    _attn_check(err, ref, f"decode_chunks_{'_'.join(map(str, past))}")


@pytest.mark.parametrize("q_lens,past", [([1], [20000]), ([1, 1, 1], [20000, 9000, 100])],
                         ids=["b1_ctx20001", "b3_ctx20001_9001_101"])
def test_attention_decode_max_chunks(lib, q_lens, past):
    """Long contexts reach the decode launcher's other shape and its chunk cap (attention.hip
    decode_shape): from 96 pages per sequence on, 4-wave workgroups; one sequence at 20001 cached
    tokens splits into MAX_DECODE_CHUNKS = 64 chunks (the last arriver merges all 64 partials, 8
    blocks of 8), three sequences into 21 each (blocks of 8, 8, 5; the 101-token sequence has only
    2 pages, so 2 of them); against fp32 SDPA with the same bounds."""
    err, ref = _attn_case(lib, 32, 8, q_lens, past, seed=11, n_pages=480)
    _attn_check(err, ref, f"decode_chunks_{'_'.join(map(str, past))}")


@pytest.mark.parametrize("H,KV", [(32, 8), (16, 8), (4, 2), (64, 8)])
def test_attention_prefill(lib, H, KV):
    """The prefill attention (4 waves x 48 query rows) on ragged prompts, with and without
    cached prefixes: a 700-token prompt (several 192-row blocks, > 4 pages) and a 1000-token
    prompt behind 300 cached tokens (masks on pages that start mid-block)."""
    err, ref = _attn_case(lib, H, KV, [1, 17, 64, 130, 700, 1000], [0, 5, 0, 200, 61, 300], seed=H + 1)
    _attn_check(err, ref, f"prefill_H{H}_KV{KV}")


def test_attention_prefill_q32b_2048(lib):
    """The Qwen3-32B head shape (64 q / 8 kv heads) on one 2048-token prompt: long softmax rows
    with many lazy rescales, the config-5 kernel path (the prefill attention's rms
    error against fp32, bounded here, not only its max)."""
    err, ref = _attn_case(lib, 64, 8, [2048], [0], seed=5)
    _attn_check(err, ref, "prefill_q32b_T2048")


def test_peak_probes_run():
    """The roofline probes (probe.hip) launch and measure plausible rates: HBM read between
    1 TB/s and the 8 TB/s spec, bf16 MFMA between 100 TF/s and the 2.5 PF/s dense spec."""
    import bench
    pk = bench.measured_peaks(torch.device(DEV, 0))
    assert 1000.0 < pk["hbm_read_GBps"] <= 8000.0, pk
    assert 100.0 < pk["mfma_bf16_TFLOPs"] <= 2500.0, pk
