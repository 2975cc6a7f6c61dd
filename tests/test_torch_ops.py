"""torch.ops.inferd (inferd_amd/csrc/torch_ops.cpp): the C-ABI registered as PyTorch-ROCm
operators, the binding runtime.py drives the engine through.  CPU: every op and class is
registered with its schema and the host-only page-table ops work and raise the library's
errors.  GPU: the runtime (torch ops) gives bit-identical hidden states, logits and greedy ids to
the same span driven through the plain ctypes binding of the C-ABI, eagerly and as a captured
decode graph."""
import pytest
import torch

SEED = 1234


def test_ops_registered_and_kv_host_ops():
    import inferd_amd.ops as O
    for name in O.OPS:
        assert hasattr(torch.ops.inferd, name), name
    assert "Tensor(b!)? next_ids" in str(torch.ops.inferd.span_forward.default._schema)
    t = torch.ops.inferd.kv_create(10)
    try:
        torch.ops.inferd.kv_reserve(t, 5, 70)
        torch.ops.inferd.kv_reserve(t, 6, 1)
        assert torch.ops.inferd.kv_query(t, 5) == (0, 2)
        torch.ops.inferd.kv_advance(t, [5, 6], 1)
        assert torch.ops.inferd.kv_query(t, 5) == (1, 2) and torch.ops.inferd.kv_query(t, 6) == (1, 1)
        with pytest.raises(RuntimeError, match="past the reserved pages"):
            torch.ops.inferd.kv_advance(t, [5], 300)
        with pytest.raises(RuntimeError, match="KV pool exhausted"):
            torch.ops.inferd.kv_reserve(t, 7, 64 * 20)
        words, shape = torch.ops.inferd.kv_build_batch(t, [5, 6], [2, 1], torch.device("cpu"))
        # [seq_start 3 | positions 3 | slots 3 | ctx_lens 2 | block table 2 x 2]
        assert shape == [2, 3, 2, 3, 2, 0]
        assert words.tolist() == [0, 2, 3, 1, 2, 1, 1, 2, 2 * 64 + 1, 3, 2, 0, 1, 2, 0]
        torch.ops.inferd.kv_release(t, 5)
        assert torch.ops.inferd.kv_query(t, 5) == (-1, 0)
    finally:
        torch.ops.inferd.kv_destroy(t)


def test_decode_graph_class_registered():
    import inferd_amd.ops as O
    for name in O.CLASSES:
        cls = getattr(torch.classes.inferd, name)
        assert cls is not None
    # its methods: graph replay, the same step launched kernel by kernel, the steps left
    names = {str(x).split("(")[0] for x in torch._C._jit_get_custom_class_schemas() if "inferd.DecodeGraph _0" in str(x)}
    assert {"__init__", "launch", "launch_eager", "steps_left"} <= names, names
    # a DecodeGraph needs a GPU device; the schema refuses a CPU one before touching a handle
    with pytest.raises(RuntimeError, match="GPU"):
        torch.classes.inferd.DecodeGraph(1, 1, [0], 1, None, None, None, None, None, torch.device("cpu"))


@pytest.mark.gpu
def test_span_through_torch_ops_matches_ctypes():
    """runtime.SpanRuntime (torch.ops.inferd / torch.classes.inferd.DecodeGraph, the node-facing
    binding) against the same span driven through the plain ctypes binding of the C-ABI (a
    non-torch host's view: inferd_kv_build_batch, inferd_span_forward, and a decode graph captured
    over inferd_kv_build_decode_batch's descriptor with no manual edits): bit-identical hidden
    states, logits and greedy ids, eagerly and over 4 graph replays.  Also: the ops refuse
    tensors too small for the batch, and a graph refuses a launch past its reserved steps."""
    import ctypes as C
    from inferd_amd import _lib
    from inferd_amd.runtime import MODELS, DecodeGraph, SpanRuntime
    d = MODELS["tiny"]
    dev = torch.device("cuda", 0)
    kw = dict(has_embed=True, has_lm_head=True, kv_pages=16, max_tokens=256, max_seqs=4, max_positions=1024)
    ref = SpanRuntime(d, 0, d.layers, device=dev, **kw)
    ref.init_synthetic(SEED)
    L = _lib.load()
    st = torch.cuda.current_stream(dev).cuda_stream
    cfg = _lib.SpanConfig(hidden=d.hidden, intermediate=d.intermediate, heads=d.heads, kv_heads=d.kv_heads,
                          head_dim=d.head_dim, vocab=d.vocab, first_layer=0, n_layers=d.layers, has_embed=1,
                          has_lm_head=1, rms_eps=d.eps, rope_theta=d.rope_theta, max_positions=1024, kv_pages=16,
                          max_tokens=256, max_seqs=4)
    h, t, g = _lib.c_p(), _lib.c_p(), _lib.c_p()
    _lib.check(L.inferd_span_create(cfg, h))
    _lib.check(L.inferd_kv_create(16, t))
    try:
        _lib.check(L.inferd_span_init_synthetic(h, SEED, st))
        got = _lib.SpanConfig()
        _lib.check(L.inferd_span_get_config(h, got))
        assert (got.hidden, got.vocab, got.n_layers, got.max_seqs) == (d.hidden, d.vocab, d.layers, 4)
        keys = (C.c_uint64 * 3)(0, 1, 2)
        prompts = torch.randint(0, d.vocab, (3, 40), generator=torch.Generator().manual_seed(3))
        for s in range(3):
            _lib.check(L.inferd_kv_reserve(t, s, 40))
        nn = (C.c_int32 * 3)(40, 40, 40)
        nw = L.inferd_kv_batch_words(t, keys, nn, 3)
        host = torch.empty(nw, dtype=torch.int32)
        words = torch.empty(nw, dtype=torch.int32, device=dev)
        b = _lib.Batch()
        _lib.check(L.inferd_kv_build_batch(t, keys, nn, 3, C.cast(host.data_ptr(), C.POINTER(C.c_int32)), nw,
                                           words.data_ptr(), b))
        words.copy_(host)
        ids = prompts.reshape(-1).to(dev, torch.int32)
        hid = torch.empty(120, d.hidden, dtype=torch.bfloat16, device=dev)
        nid = torch.empty(3, dtype=torch.int32, device=dev)
        lg = torch.empty(3, d.vocab, dtype=torch.bfloat16, device=dev)
        _lib.check(L.inferd_span_forward(h, b, ids.data_ptr(), None, hid.data_ptr(), nid.data_ptr(), lg.data_ptr(),
                                         None, st))
        _lib.check(L.inferd_kv_advance_many(t, keys, 3, 40))
        out = ref.forward([(f"s{s}", 40) for s in range(3)], ids=prompts.reshape(-1), want_hidden=True,
                          want_next_ids=True, want_logits=True)
        assert torch.equal(hid.cpu(), out["hidden"].cpu())
        assert torch.equal(lg.cpu(), out["logits"].cpu()) and torch.equal(nid.cpu(), out["next_ids"].cpu())
        # the ops check every buffer against the batch shape and the span's sizes
        bt = ref.build_batch([(ref._seq("s0"), 1)])
        with pytest.raises(RuntimeError, match="elements"):
            torch.ops.inferd.span_forward(ref.handle, bt.words, bt.shape, ids[:1], None,
                                          torch.empty(1, dtype=torch.bfloat16, device=dev), None, None)
        with pytest.raises(RuntimeError, match="logits"):
            torch.ops.inferd.span_lm_head(ref.handle, hid[:4], torch.empty(4, dtype=torch.bfloat16, device=dev))
        # 4 decode steps: ctypes capture over the native decode descriptor vs the torch DecodeGraph
        nw = L.inferd_kv_decode_batch_words(t, keys, 3, 4)
        host = torch.empty(nw, dtype=torch.int32)
        words2 = torch.empty(nw, dtype=torch.int32, device=dev)
        b2 = _lib.Batch()
        _lib.check(L.inferd_kv_build_decode_batch(t, keys, 3, 4, C.cast(host.data_ptr(), C.POINTER(C.c_int32)), nw,
                                                  words2.data_ptr(), b2))
        assert (b2.n_seqs, b2.n_tokens, b2.max_q_len, b2.max_ctx_len, b2.decode) == (3, 3, 1, 44, 1)
        assert host[10:13].tolist() == [40, 40, 40]           # ctx_lens = the cached lengths
        words2.copy_(host)
        cur = nid.clone()
        cs = torch.cuda.Stream(dev)
        cs.wait_stream(torch.cuda.current_stream(dev))
        _lib.check(L.inferd_span_graph_capture(h, b2, 1, cur.data_ptr(), None, None, cur.data_ptr(), None,
                                               cs.cuda_stream, g))
        torch.cuda.current_stream(dev).wait_stream(cs)
        ref_ids = out["next_ids"].clone()
        rg = DecodeGraph(ref, [f"s{s}" for s in range(3)], 4, ids=ref_ids, next_ids=ref_ids)
        for _ in range(4):
            _lib.check(L.inferd_graph_launch(g, st))
            _lib.check(L.inferd_kv_advance_many(t, keys, 3, 1))
            rg.launch()
            torch.cuda.synchronize()
            assert torch.equal(cur.cpu(), ref_ids.cpu())
        assert rg.launched == 4
        with pytest.raises(RuntimeError, match="ran out of reserved steps"):
            rg.launch()
        ln, npg = C.c_int32(), C.c_int32()
        _lib.check(L.inferd_kv_query(t, 0, C.byref(ln), C.byref(npg)))
        assert (ln.value, npg.value) == (44, 1) and ref.kv.query(ref._seq("s0").seq) == (44, 1)
        ref.check_errors()
    finally:
        if g.value:
            L.inferd_graph_destroy(g)
        L.inferd_kv_destroy(t)
        L.inferd_span_destroy(h)
