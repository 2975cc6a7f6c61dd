"""CPU tests of the host side: the C-ABI library exports, the drop-in module surface and
wire codec, the offline splitter, the KV page pool and the batch descriptors."""
import ctypes
import json
import os
import re

import numpy as np
import pytest
import torch

from golden_io import GOLDEN

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_functions():
    src = open(os.path.join(ROOT, "include", "inferd_span.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(inferd_\w+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    from inferd_amd import _lib
    lib = ctypes.CDLL(_lib.LIB_PATH)
    names = _header_functions()
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    # and the Python binding declares a signature for every one of them
    assert sorted(_lib.SIGNATURES) == names


def test_library_loads_and_reports_version():
    from inferd_amd import _lib
    lib = _lib.load()
    assert lib.inferd_abi_version() == _lib.ABI_VERSION == 5
    # error path without a GPU: a null config is rejected with a message
    h = _lib.c_p()
    rc = lib.inferd_span_create(None, h)
    assert rc == 1 and b"null" in lib.inferd_last_error()


def test_io_elems_matches_the_pipeline_record_sizes():
    """inferd_span_io_elems (the C-ABI's buffer-size rule, a pure function of the config; no GPU)
    agrees with the host's hand-off sizes (pipeline.buffer_elems) at every boundary kind and with
    the final_norm_out rows, for prefill, gemv-sized and decode calls."""
    from inferd_amd import _lib
    from inferd_amd.pipeline import buffer_elems
    from inferd_amd.runtime import MODELS
    lib = _lib.load()
    d = MODELS["qwen3-8b"]
    base = dict(hidden=d.hidden, intermediate=d.intermediate, heads=d.heads, kv_heads=d.kv_heads,
                head_dim=d.head_dim, vocab=d.vocab, first_layer=0, n_layers=2, max_seqs=16)
    kinds = {"layer": {}, "gateup": dict(gateup_split_first=4096, gateup_split_last=4096),
             "o": dict(o_split_first=1, o_split_last=1), "q": dict(qkv_split_first=1, qkv_split_last=1)}
    for kind, kw in kinds.items():
        cfg = _lib.SpanConfig(**base, **kw)
        for rows, decode in ((1, 1), (5, 1), (16, 1), (48, 0), (64, 0), (65, 0), (300, 0)):
            want = buffer_elems(d, rows, 4096 if kind == "gateup" else 0, kind == "o", bool(decode), kind == "q")
            for which in (0, 1):
                got = lib.inferd_span_io_elems(ctypes.byref(cfg), rows, rows if decode else 1, decode, which)
                assert got == want, (kind, rows, decode, which, got, want)
    cfg = _lib.SpanConfig(**base, final_norm_out=1)
    assert lib.inferd_span_io_elems(ctypes.byref(cfg), 5, 5, 1, 1) == 16 * d.hidden
    assert lib.inferd_span_io_elems(ctypes.byref(cfg), 5, 5, 1, 0) == 5 * d.hidden
    assert lib.inferd_span_io_elems(None, 5, 5, 1, 0) == -1 and b"io_elems" in lib.inferd_last_error()
    assert lib.inferd_span_io_elems(ctypes.byref(cfg), 5, 5, 1, 2) == -1


def test_codec_matches_reference_fixture():
    from inferd_amd.partitioned_models import base64_to_tensor, build_decoder_attention_mask, tensor_to_base64
    g = json.load(open(os.path.join(GOLDEN, "codec.json")))
    t = torch.tensor(g["input"], dtype=torch.float32).reshape(g["shape"])
    assert tensor_to_base64(t) == g["meta"]                 # byte-identical wire format (fp32)
    assert torch.equal(base64_to_tensor(g["meta"]), t)
    m = build_decoder_attention_mask(torch.tensor([[1, 1, 1, 0, 1]]))
    assert m.to(torch.int32).reshape(-1).tolist() == g["mask"] and list(m.shape) == g["mask_shape"]


def test_codec_bf16_roundtrip():
    from inferd_amd.partitioned_models import base64_to_tensor, tensor_to_base64
    t = torch.randn(1, 7, 33).to(torch.bfloat16)
    meta = tensor_to_base64(t)
    assert meta["dtype"] == "bfloat16" and meta["shape"] == [1, 7, 33]
    back = base64_to_tensor(json.loads(json.dumps(meta)))
    assert back.dtype == torch.bfloat16 and torch.equal(back, t)


def test_module_surface_matches_reference():
    """run_node.py:6 imports FirstStage/StageInner/LastStage; task.py builds PartitionedQwen2."""
    import inferd_amd.partitioned_models as P
    for name in ("FirstStage", "StageInner", "LastStage", "PartitionedQwen2", "tensor_to_base64",
                 "base64_to_tensor", "build_decoder_attention_mask"):
        assert hasattr(P, name)
    import inspect
    assert list(inspect.signature(P.PartitionedQwen2.__init__).parameters)[1:] == \
        ["model_name", "num_stages", "stage", "parts_path"]
    assert list(inspect.signature(P.PartitionedQwen2.forward).parameters)[1:] == ["inputs"]


def test_kv_table_and_batch_descriptor():
    """The native page table (inferd_kv_*, kvtable.hip; host-only calls, no GPU): reserve /
    advance / release, lowest-page-first allocation, all-or-nothing exhaustion, and the batch
    descriptor words of a cached continuation plus a fresh sequence."""
    from inferd_amd.runtime import KvTable
    kv = KvTable(10)
    kv.reserve(1, 73)     # sequence a: 70 cached tokens + 3 new -> 2 pages
    kv.advance(1, 70)
    kv.reserve(2, 5)      # sequence b: 5 new tokens -> 1 page
    assert kv.pages(1) == [0, 1] and kv.pages(2) == [2] and kv.n_free == 7
    assert kv.query(1) == (70, 2) and kv.query(3) == (-1, 0)
    batch = kv.build_batch([(1, 3), (2, 5)], "cpu")
    assert (batch.n_seqs, batch.n_tokens, batch.max_q_len, batch.max_ctx_len, batch.decode) == (2, 8, 5, 73, 0)
    w = batch.words.tolist()
    assert w[0:3] == [0, 3, 8]                                       # seq_start
    assert w[3:11] == [70, 71, 72, 0, 1, 2, 3, 4]                    # positions
    assert w[11:19] == [1 * 64 + 6, 1 * 64 + 7, 1 * 64 + 8] + [2 * 64 + i for i in range(5)]  # slots
    assert w[19:21] == [73, 5]                                       # ctx_lens
    assert w[21:25] == [0, 1, 2, 0] and len(w) == 25                 # block table
    # the same descriptor through the ctypes binding (the non-torch host's view)
    from inferd_amd import _lib
    cb = _lib.batch_struct(batch.words, batch.shape)

    def arr(ptr, n):
        return list((ctypes.c_int32 * n).from_address(ptr))
    assert arr(cb.seq_start, 3) == [0, 3, 8] and arr(cb.block_table, 4) == [0, 1, 2, 0]
    assert cb.seq_start == batch.words.data_ptr()
    with pytest.raises(RuntimeError, match="KV pool exhausted"):
        kv.reserve(3, 8 * 64)
    assert kv.n_free == 7 and kv.query(3)[1] == 0          # nothing taken
    with pytest.raises(RuntimeError):
        kv.build_batch([(1, 3), (1, 3)], "cpu")             # a sequence twice
    with pytest.raises(RuntimeError):
        kv.build_batch([(2, 65)], "cpu")                    # pages not reserved
    with pytest.raises(RuntimeError):
        kv.advance(2, 65)                                   # past the reserved pages
    # a decode-graph replay's host advance: one native call for the whole batch, all or nothing
    kv.advance_many([1, 2], 3)
    assert kv.query(1)[0] == 73 and kv.query(2)[0] == 3
    with pytest.raises(RuntimeError, match="past the reserved pages"):
        kv.advance_many([1, 2], 62)                                     # sequence a: past its 2 pages
    assert kv.query(1)[0] == 73 and kv.query(2)[0] == 3                 # nothing advanced
    with pytest.raises(RuntimeError, match="only once"):
        kv.advance_many([2, 2], 1)                                      # a sequence twice
    kv.release(1)
    assert kv.n_free == 9
    kv.reserve(4, 64)                                       # a's first page comes back first
    assert kv.pages(4) == [0]
    kv.release(99)                                          # absent: no-op


def test_split_model_writes_stage_files(tmp_path):
    """Offline splitter: roles from `stage` vs stages_count (not list order), metadata, keys."""
    from safetensors import safe_open
    from inferd_amd.runtime import MODELS
    from inferd_amd.split_model import split
    from oracle import qwen3_ref as R
    d = R.CONFIGS["tiny"]
    cfg = {"model_name": "tiny", "parts_dir": str(tmp_path), "stages_count": 3,
           "stages": [{"name": "node0", "stage": 0, "start_layer": 0, "end_layer": 0},
                      {"name": "node1", "stage": 1, "start_layer": 1, "end_layer": 2},
                      {"name": "node2", "stage": 2, "start_layer": 3, "end_layer": 3},
                      {"name": "node3", "stage": 2, "start_layer": 3, "end_layer": 3}]}
    glob = R.gen_global_weights(d, 1234)

    def get_layer(i):
        W = R.gen_layer_weights(d, 1234, i)
        return {("self_attn." if k in ("q_proj", "k_proj", "v_proj", "o_proj", "q_norm", "k_norm") else
                 "mlp." if k in ("gate_proj", "up_proj", "down_proj") else "") + k + ".weight": v
                for k, v in W.items()}
    paths = split(cfg, MODELS["tiny"], get_layer, lambda n: glob[n])
    assert len(paths) == 4
    with safe_open(paths[2], framework="pt") as f:   # node2: stage 2 of 3 -> LastStage
        meta = f.metadata()
        assert meta["last"] == "1" and meta["first"] == "0"
        assert "lm_head.weight" in f.keys() and "layers.0.mlp.down_proj.weight" in f.keys()
    with safe_open(paths[1], framework="pt") as f:
        assert f.metadata()["start_layer"] == "1" and f.metadata()["end_layer"] == "2"
        assert torch.equal(f.get_tensor("layers.1.self_attn.q_proj.weight"), R.gen_layer_weights(d, 1234, 2)["q_proj"])
        assert "embed.weight" not in f.keys()


def test_weightgen_numpy_known_values():
    """Pin the generator definition itself (splitmix64 reference values)."""
    from oracle import weightgen as wg
    z = wg.splitmix64(np.array([0, 1, 0xFFFFFFFFFFFFFFFF], dtype=np.uint64))
    # splitmix64 published test vector: seed 0 -> 0xE220A8397B1DCDAF
    assert int(z[0]) == 0xE220A8397B1DCDAF
    v = wg.uniform_fp32(1234, 7, 5, 1.0)
    assert v.dtype == np.float32 and np.all(np.abs(v) <= 1.0)


def test_weightgen_c_matches_numpy():
    """The oracle's C generator (oracle/weightgen.c, what the 8B / 32B oracle runs use) gives
    the numpy definition's bf16 bits exactly: linear and norm tensors, a global tensor id, an
    odd length."""
    import subprocess
    from oracle import weightgen as wg
    if wg.c_generator() is None:
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
        wg._CLIB = None
    assert wg.c_generator() is not None
    for seed, tid, shape, name in [(1234, 3 * 16 + 8, (512, 4096), "gate_proj"), (1234, 7, (4096,), "input_layernorm"),
                                   (99, 0xFFFF0002, (1000, 256), "lm_head"), (5, 17, (12345,), "q_proj")]:
        a = wg.gen_tensor_bf16_bits(seed, tid, shape, name, use_c=False)
        b = wg.gen_tensor_bf16_bits(seed, tid, shape, name)
        assert np.array_equal(a, b), (tid, name)


def _brute_split(n_layers, n, lc, hc):
    """All compositions of n_layers into n positive parts; (max, sum sq) optimum."""
    import itertools
    best = None
    for cuts in itertools.combinations(range(1, n_layers), n - 1):
        b = (0,) + cuts + (n_layers,)
        sizes = [b[i + 1] - b[i] for i in range(n)]
        costs = [k * lc + (hc if i == n - 1 else 0.0) for i, k in enumerate(sizes)]
        key = (max(costs), sum(c * c for c in costs))
        if best is None or key < best[0]:
            best = (key, sizes)
    return best


@pytest.mark.parametrize("n_layers,n,hc", [(12, 3, 2.4), (12, 4, 0.0), (10, 2, 5.0), (9, 9, 1.0), (13, 5, 3.3)])
def test_balanced_split_is_min_max(n_layers, n, hc):
    from inferd_amd.pipeline import balanced_split
    spans = balanced_split(n_layers, n, 1.0, hc)
    sizes = [k for _, k in spans]
    assert sum(sizes) == n_layers and min(sizes) >= 1
    assert [f for f, _ in spans] == [sum(sizes[:i]) for i in range(n)]
    costs = [k + (hc if i == n - 1 else 0.0) for i, k in enumerate(sizes)]
    (bmax, bsq), _ = _brute_split(n_layers, n, 1.0, hc)
    assert max(costs) == pytest.approx(bmax) and sum(c * c for c in costs) == pytest.approx(bsq)


def test_bench_stage_split_qwen3_8b():
    """bench.py's default stage split is BASELINE config 3's even split ([18,18] / [9,9,9,9] /
    [5,5,5,5,4,4,4,4]); `balanced` prices the lm_head on the last stage: its slowest stage is 5
    layers at N = 8 where the even split's is 4 layers + lm_head."""
    import bench
    from inferd_amd.runtime import MODELS
    d = MODELS["qwen3-8b"]
    assert [k for _, k in bench.stage_split(d, 8, 16, 2048)] == [5, 5, 5, 5, 4, 4, 4, 4]
    assert [k for _, k in bench.stage_split(d, 2, 16, 2048)] == [18, 18]
    assert [k for _, k in bench.stage_split(d, 4, 16, 2048)] == [9, 9, 9, 9]
    assert [k for _, k in bench.stage_split(d, 8, 16, 2048, "balanced")] == [4, 5, 5, 5, 5, 5, 5, 2]
    assert [k for _, k in bench.stage_split(d, 1, 16, 2048)] == [36]


def test_build_decode_batch_descriptor():
    """inferd_kv_build_decode_batch (the descriptor a decode graph is captured on, advance = 1):
    reserves n_steps more tokens per sequence all or nothing, positions / slots start at 0 (the
    graph's scheduler step writes them), ctx_lens = the cached lengths, max_ctx_len = capacity."""
    import ctypes as C
    from inferd_amd import _lib
    L = _lib.load()
    t = _lib.c_p()
    _lib.check(L.inferd_kv_create(12, t))
    try:
        for seq, n in ((5, 70), (6, 10)):
            _lib.check(L.inferd_kv_reserve(t, seq, n))
            _lib.check(L.inferd_kv_advance(t, seq, n))
        keys = (C.c_uint64 * 2)(5, 6)
        nw = L.inferd_kv_decode_batch_words(t, keys, 2, 60)
        assert nw == 3 + 2 + 2 + 2 + 2 * 3          # max pages after the reservation: 3 (130 tokens)
        host = (C.c_int32 * nw)()
        b = _lib.Batch()
        _lib.check(L.inferd_kv_build_decode_batch(t, keys, 2, 60, host, nw, None, b))
        assert (b.n_seqs, b.n_tokens, b.max_q_len, b.max_ctx_len, b.max_pages, b.decode) == (2, 2, 1, 130, 3, 1)
        w = list(host)
        assert w[0:3] == [0, 1, 2] and w[3:5] == [0, 0] and w[5:7] == [0, 0]   # seq_start, positions, slots
        assert w[7:9] == [70, 10]                                               # ctx_lens = cached lengths
        assert w[9:12] == [0, 1, 3] and w[12:15] == [2, 4, 0]                   # block table (pages in order)
        ln, npg = C.c_int32(), C.c_int32()
        _lib.check(L.inferd_kv_query(t, 5, C.byref(ln), C.byref(npg)))
        assert (ln.value, npg.value) == (70, 3)                                 # reserved, not advanced
        # all or nothing: 512 more tokens of both sequences need 14 pages, 7 are free
        free = C.c_int32()
        _lib.check(L.inferd_kv_free_pages(t, C.byref(free)))
        assert L.inferd_kv_build_decode_batch(t, keys, 2, 64 * 8, host, nw, None, b) == _lib.INFERD_ERR_ARG  # buffer
        big = L.inferd_kv_decode_batch_words(t, keys, 2, 64 * 8)
        hb = (C.c_int32 * big)()
        assert L.inferd_kv_build_decode_batch(t, keys, 2, 64 * 8, hb, big, None, b) == _lib.INFERD_ERR_NOMEM
        free2 = C.c_int32()
        _lib.check(L.inferd_kv_free_pages(t, C.byref(free2)))
        assert free2.value == free.value                                        # nothing taken
        assert L.inferd_kv_decode_batch_words(t, (C.c_uint64 * 1)(99), 1, 1) == -1   # unknown sequence
    finally:
        L.inferd_kv_destroy(t)


def test_build_batch_descriptor_layout():
    """The native batch builder (inferd_kv_build_batch) against a per-token restatement of
    the descriptor: seq_start | positions | slots (page * 64 + offset) | ctx_lens | block
    table, over random reserve / advance / release histories (scattered page lists)."""
    import random
    from inferd_amd.runtime import KV_PAGE, KvTable
    rng = random.Random(0)
    kv = KvTable(4096)
    live = {}
    for it in range(100):
        for _ in range(rng.randint(0, 3)):                  # churn: scatter the free list
            if live and rng.random() < 0.5:
                kv.release(live.pop(rng.choice(list(live))))
        seqs = []
        for _b in range(rng.randint(1, 6)):
            key = 1000 * it + _b
            past, n = rng.randint(0, 300), rng.randint(1, 200)
            kv.reserve(key, past + n + rng.randint(0, 100))
            kv.advance(key, past)
            live[key] = key
            seqs.append((key, n))
        batch = kv.build_batch(seqs, "cpu")
        dev = batch.words
        pages = {k: kv.pages(k) for k, _ in seqs}
        max_pages = max(len(pages[k]) for k, _ in seqs)
        start, pos, slots, ctx, table = [0], [], [], [], []
        for k, n in seqs:
            past = kv.query(k)[0]
            for i in range(n):
                p = past + i
                pos.append(p)
                slots.append(pages[k][p // KV_PAGE] * KV_PAGE + p % KV_PAGE)
            start.append(start[-1] + n)
            ctx.append(past + n)
            table += pages[k] + [0] * (max_pages - len(pages[k]))
        assert dev.tolist() == start + pos + slots + ctx + table
        assert batch.n_tokens == sum(n for _, n in seqs) and batch.max_ctx_len == max(ctx)
        assert batch.max_q_len == max(n for _, n in seqs) and batch.max_pages == max_pages
        for k, _ in seqs:
            if rng.random() < 0.7:
                kv.release(live.pop(k))


def test_split_model_from_hf_checkpoint(tmp_path):
    """split_model's HF-safetensors source (sharded checkpoint dir, split_model.py:81's
    from_pretrained weights): every stage file holds the checkpoint's tensors under the
    engine's keys, roles from `stage`."""
    from safetensors import safe_open
    from hf_fixtures import write_hf_checkpoint
    from inferd_amd.runtime import MODELS
    from inferd_amd.split_model import hf_checkpoint_source, split
    from oracle import qwen3_ref as R
    d = R.CONFIGS["tiny"]
    ck = write_hf_checkpoint(str(tmp_path / "hf"), d, 99)
    cfg = {"model_name": "tiny", "parts_dir": str(tmp_path / "out"), "stages_count": 2,
           "stages": [{"name": "node0", "stage": 0, "start_layer": 0, "end_layer": 1},
                      {"name": "node1", "stage": 1, "start_layer": 2, "end_layer": 3}]}
    paths = split(cfg, MODELS["tiny"], *hf_checkpoint_source(ck))
    g = R.gen_global_weights(d, 99)
    with safe_open(paths[0], framework="pt") as f:
        assert torch.equal(f.get_tensor("embed.weight"), g["embed_tokens"]) and "lm_head.weight" not in f.keys()
        assert torch.equal(f.get_tensor("layers.1.mlp.up_proj.weight"), R.gen_layer_weights(d, 99, 1)["up_proj"])
    with safe_open(paths[1], framework="pt") as f:
        assert torch.equal(f.get_tensor("lm_head.weight"), g["lm_head"]) and f.metadata()["last"] == "1"
        assert torch.equal(f.get_tensor("layers.0.self_attn.k_norm.weight"), R.gen_layer_weights(d, 99, 2)["k_norm"])


def test_convert_reference_parts_executes_nothing(tmp_path):
    """The reference's pickled stage modules (torch.save(module), split_model.py:107) convert
    to engine stage files through the inert unpickler: tensors identical, every class the
    pickle names stays a stub -- including one whose __setstate__ would record a call."""
    import pickle
    from safetensors import safe_open
    import hf_fixtures
    from inferd_amd import convert_parts as C
    from inferd_amd.runtime import MODELS
    from oracle import qwen3_ref as R
    d = R.CONFIGS["tiny"]
    cfg = {"model_name": "tiny", "parts_dir": str(tmp_path / "parts"), "stages_count": 3,
           "stages": [{"name": "a", "stage": 0, "start_layer": 0, "end_layer": 0},
                      {"name": "b", "stage": 1, "start_layer": 1, "end_layer": 2},
                      {"name": "c", "stage": 2, "start_layer": 3, "end_layer": 3}]}
    hf_fixtures.write_reference_parts(cfg["parts_dir"], cfg, d, 5)
    calls = []
    hf_fixtures.StageInner.__setstate__ = lambda self, st: calls.append(st)   # would run under torch.load
    try:
        paths = C.convert(cfg, MODELS["tiny"], cfg["parts_dir"], str(tmp_path / "out"))
        tree = C.load_inert(str(tmp_path / "parts" / "b" / "model.pth"))
    finally:
        del hf_fixtures.StageInner.__setstate__
    assert not calls and isinstance(tree, C.Stub) and tree.qualname.endswith("StageInner")
    with safe_open(paths[1], framework="pt") as f:
        assert sorted(f.keys()) == sorted(f"layers.{j}.{k}" for j in range(2) for k in C._LAYER_LEAVES)
        assert torch.equal(f.get_tensor("layers.1.self_attn.o_proj.weight"), R.gen_layer_weights(d, 5, 2)["o_proj"])
    with safe_open(paths[2], framework="pt") as f:
        assert torch.equal(f.get_tensor("lm_head.weight"), R.gen_global_weights(d, 5)["lm_head"])
    with safe_open(paths[0], framework="pt") as f:
        assert torch.equal(f.get_tensor("embed.weight"), R.gen_global_weights(d, 5)["embed_tokens"])
    with pytest.raises(pickle.UnpicklingError):    # no real class can be reconstructed
        C._reconstructor(dict, object)


def test_grpc_blob_codec_and_messages():
    """TensorBlob payloads: the reference's torch.save bytes (read weights-only) and the raw
    form round-trip every dtype the client sends; the message classes serialise with the
    reference's field numbers (qwen3.proto:5-20)."""
    from inferd_amd import grpc_span as G
    for t in (torch.randn(1, 3, 8).to(torch.bfloat16), torch.randn(2, 5), torch.arange(7),
              torch.zeros(1, 1, 4, 4, dtype=torch.bool), torch.randn(1, 1, 1, 1).to(torch.bfloat16)):
        for raw in (False, True):
            b = G.tensor_to_blob(t, raw)
            assert G.blob_is_raw(b) == raw
            back = G.blob_to_tensor(b)
            assert back.dtype == t.dtype and torch.equal(back, t)
    req = G.LayerRequest(hidden_states=G.TensorBlob(data=b"xy"), session_id="s")
    wire = req.SerializeToString()
    assert wire == b"\n\x04\n\x02xy2\x01s"     # field 1 (message: field 1 bytes), field 6 string
    assert G.LayerRequest.FromString(wire).session_id == "s"


def test_peaked_profile_oracle_definition():
    """The peaked synthetic profile: embed scaled by a power of two (exact), lm_head row p(t)
    = random row + LM_MIX * embed[t], p a bijection of the vocabulary."""
    import numpy as np
    from oracle import qwen3_ref as R
    from oracle import weightgen as wg
    d = R.CONFIGS["tiny"]
    p = wg.peaked_perm(d.vocab)
    assert sorted(p.tolist()) == list(range(d.vocab))
    g, q = R.gen_global_weights(d, 3), R.gen_global_weights(d, 3, profile="peaked")
    assert torch.equal(q["embed_tokens"].float(), g["embed_tokens"].float() * wg.EMBED_BOOST)
    t = 17
    assert torch.equal(q["lm_head"][int(p[t])], (g["lm_head"][int(p[t])].float() + wg.LM_MIX *
                                                  g["embed_tokens"][t].float()).to(torch.bfloat16))
    assert torch.equal(q["norm"], g["norm"]) and np.all(np.diff(np.sort(p)) == 1)


def test_node_group_split_and_stage_range():
    """A grouped stage's layers are split by decode bytes with the lm_head on the last rank."""
    from inferd_amd.node_group import group_split, stage_range
    from inferd_amd.runtime import MODELS
    d, s, e, prof = stage_range("synthetic:1:qwen3-8b:0:17:peaked", "x", 2, 0)
    assert (d.name, s, e, prof) == ("qwen3-8b", 0, 17, "peaked")
    sp = group_split(MODELS["qwen3-8b"], 18, 4, lm_head=True)
    sizes = [n for _, n in sp]
    assert sum(sizes) == 18 and sizes[-1] < sizes[0]
    assert [n for _, n in group_split(MODELS["qwen3-8b"], 18, 3, lm_head=False)] == [6, 6, 6]


def test_c_host_kv_table(tmp_path):
    """A plain-C host of the KV page table (tests/c_abi/kv_host.c): builds against
    include/inferd_span.h with gcc, links libinferd_span.so, runs on the CPU."""
    import shutil
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib_dir = os.path.join(root, "inferd_amd")
    if not os.path.exists(os.path.join(lib_dir, "libinferd_span.so")):
        pytest.skip("libinferd_span.so not built")
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    exe = str(tmp_path / "kv_host")
    subprocess.run([cc, "-std=c11", "-Wall", "-Werror", "-I", os.path.join(root, "include"),
                    os.path.join(root, "tests", "c_abi", "kv_host.c"), "-L", lib_dir, "-linferd_span",
                    f"-Wl,-rpath,{lib_dir}", "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "C HOST OK" in r.stdout, r.stdout + r.stderr


def test_c_host_span_builds(tmp_path):
    """The plain-C GPU host of the span engine (tests/c_abi/span_host.c; run against the GPU by
    tests/test_gpu_span.py::test_c_host_span_greedy) compiles warning-free against
    include/inferd_span.h and HIP's C API with gcc, links libinferd_span.so, and refuses a bad
    command line before touching a device."""
    import shutil
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib_dir = os.path.join(root, "inferd_amd")
    if not os.path.exists(os.path.join(lib_dir, "libinferd_span.so")):
        pytest.skip("libinferd_span.so not built")
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None or not os.path.exists("/opt/rocm/include/hip/hip_runtime_api.h"):
        pytest.skip("no C compiler / HIP headers")
    exe = str(tmp_path / "span_host")
    subprocess.run([cc, "-std=c11", "-Wall", "-Werror", "-D__HIP_PLATFORM_AMD__", "-I", os.path.join(root, "include"),
                    "-I", "/opt/rocm/include", os.path.join(root, "tests", "c_abi", "span_host.c"), "-L", lib_dir,
                    "-linferd_span", "-L", "/opt/rocm/lib", "-lamdhip64", f"-Wl,-rpath,{lib_dir}",
                    "-Wl,-rpath,/opt/rocm/lib", "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "usage" in r.stderr, r.stdout + r.stderr


def test_split_model_checkpoint_config_dims_and_refusals(tmp_path):
    """A HF checkpoint's config.json gives the stage files their geometry (any Qwen3 size, not only
    runtime.MODELS's), and checkpoints the engine cannot run are refused with the reason: a Qwen2
    config (the reference's default Qwen/Qwen2-0.5B), 64-dim heads, rope scaling, biased
    projections."""
    import json
    from dataclasses import asdict
    from safetensors import safe_open
    from safetensors.torch import save_file
    from hf_fixtures import write_hf_checkpoint
    from inferd_amd.runtime import MODELS
    from inferd_amd.split_model import checkpoint_dims, hf_checkpoint_source, split
    from oracle import qwen3_ref as R
    d = R.CONFIGS["tiny"]
    ck = write_hf_checkpoint(str(tmp_path / "hf"), d, 7)
    assert checkpoint_dims(ck) is None          # no config.json: the caller's dims
    conf = {"model_type": "qwen3", "hidden_size": d.hidden, "intermediate_size": d.intermediate,
            "num_attention_heads": d.heads, "num_key_value_heads": d.kv_heads, "num_hidden_layers": d.layers,
            "vocab_size": d.vocab, "head_dim": 128, "rms_norm_eps": 1e-6, "rope_theta": 1000000.0,
            "max_position_embeddings": 40960, "attention_bias": False, "rope_scaling": None}
    with open(tmp_path / "hf" / "config.json", "w") as f:
        json.dump(conf, f)
    dims = checkpoint_dims(ck, name="tiny")
    assert asdict(dims) == asdict(MODELS["tiny"])
    cfg = {"model_name": "tiny", "parts_dir": str(tmp_path / "out"), "stages_count": 1,
           "stages": [{"name": "n0", "stage": 0, "start_layer": 0, "end_layer": d.layers - 1}]}
    (path,) = split(cfg, dims, *hf_checkpoint_source(ck))
    with safe_open(path, framework="pt") as f:
        assert json.loads(f.metadata()["dims"]) == asdict(dims)
    for bad, why in (({"model_type": "qwen2", "head_dim": 64}, "qwen2"), ({"head_dim": 64}, "head_dim"),
                     ({"rope_scaling": {"type": "yarn", "factor": 4.0}}, "rope_scaling"),
                     ({"attention_bias": True}, "attention_bias")):
        with open(tmp_path / "hf" / "config.json", "w") as f:
            json.dump({**conf, **bad}, f)
        with pytest.raises(ValueError, match=why):
            checkpoint_dims(ck)
    save_file({"model.layers.0.self_attn.q_proj.bias": torch.zeros(4)}, str(tmp_path / "hf" / "bias.safetensors"))
    with pytest.raises(ValueError, match="biased"):
        hf_checkpoint_source(ck)
