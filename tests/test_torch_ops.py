"""torch.ops.inferd (inferd_amd/csrc/torch_ops.cpp): the C-ABI registered as PyTorch-ROCm
operators.  CPU: every op is registered with its schema and the host-only page-table ops work
and raise the library's errors.  GPU: a span driven entirely through torch.ops gives
bit-identical hidden states, logits and greedy ids to the same span driven through the ctypes
binding (inferd_amd/runtime.py), eagerly and as a captured decode graph."""
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


@pytest.mark.gpu
def test_span_through_torch_ops_matches_ctypes():
    import inferd_amd.ops as O
    from inferd_amd.runtime import MODELS, DecodeGraph, SpanRuntime
    d = MODELS["tiny"]
    dev = torch.device("cuda", 0)
    kw = dict(has_embed=True, has_lm_head=True, kv_pages=16, max_tokens=256, max_seqs=4, max_positions=1024)
    ref = SpanRuntime(d, 0, d.layers, device=dev, **kw)
    ref.init_synthetic(SEED, "peaked")
    cfg = O.span_config(d, 0, d.layers, **kw)
    span = torch.ops.inferd.span_create(cfg, d.eps, d.rope_theta, dev)
    table = torch.ops.inferd.kv_create(16)
    try:
        # peaked profile = synthetic layers + the composed embed / lm_head, set through the op
        torch.ops.inferd.span_init_synthetic(span, SEED, dev)
        emb = torch.empty(d.vocab, d.hidden, dtype=torch.bfloat16, device=dev)
        lm = torch.empty_like(emb)
        from inferd_amd import runtime as RT
        e0 = RT.gen_tensor(SEED, RT.GLOBAL_TENSOR_IDS["embed_tokens"], (d.vocab, d.hidden), False, dev).float()
        l0 = RT.gen_tensor(SEED, RT.GLOBAL_TENSOR_IDS["lm_head"], (d.vocab, d.hidden), False, dev).float()
        perm = (torch.arange(d.vocab, device=dev) * RT.PERM_MUL + RT.PERM_ADD) % d.vocab
        l0[perm] += RT.LM_MIX * e0
        emb.copy_((e0 * RT.EMBED_BOOST).to(torch.bfloat16))
        lm.copy_(l0.to(torch.bfloat16))
        torch.ops.inferd.span_set_weight(span, -1, "embed_tokens", emb)
        torch.ops.inferd.span_set_weight(span, -1, "lm_head", lm)
        g = torch.Generator().manual_seed(3)
        prompts = torch.randint(0, d.vocab, (3, 40), generator=g)
        # prefill: 3 sequences of 40 tokens
        for s in range(3):
            torch.ops.inferd.kv_reserve(table, s, 40)
        words, shape = torch.ops.inferd.kv_build_batch(table, [0, 1, 2], [40, 40, 40], dev)
        ids = prompts.reshape(-1).to(dev, torch.int32)
        hid = torch.empty(120, d.hidden, dtype=torch.bfloat16, device=dev)
        nid = torch.empty(3, dtype=torch.int32, device=dev)
        lg = torch.empty(3, d.vocab, dtype=torch.bfloat16, device=dev)
        torch.ops.inferd.span_forward(span, words, shape, ids, None, hid, nid, lg)
        torch.ops.inferd.kv_advance(table, [0, 1, 2], 40)
        out = ref.forward([(f"s{s}", 40) for s in range(3)], ids=prompts.reshape(-1), want_hidden=True,
                          want_next_ids=True, want_logits=True)
        assert torch.equal(hid.cpu(), out["hidden"].cpu())
        assert torch.equal(lg.cpu(), out["logits"].cpu()) and torch.equal(nid.cpu(), out["next_ids"].cpu())
        # 4 decode steps as a captured graph through the ops vs the ctypes DecodeGraph
        for s in range(3):
            torch.ops.inferd.kv_reserve(table, s, 4)
        words, shape = torch.ops.inferd.kv_build_batch(table, [0, 1, 2], [1, 1, 1], dev)
        shape = list(shape)
        shape[3] = 44                                        # max_ctx_len = the capacity (header: advance = 1)
        # the graph's scheduler step writes position = ctx_lens[b]: start the descriptor at 40
        cur = nid.clone()
        gr = torch.ops.inferd.graph_capture(span, words, shape, cur, None, None, cur, None)
        ref_ids = out["next_ids"].clone()
        rg = DecodeGraph(ref, [f"s{s}" for s in range(3)], 4, ids=ref_ids, next_ids=ref_ids)
        n = (3 + 1) + 3 + 3 + 3 + 3 * shape[4]             # [seq_start | positions | slots | ctx_lens | table]
        words[10:13] = 40                                    # ctx_lens = the cached length before the first replay
        for _ in range(4):
            torch.ops.inferd.graph_launch(gr, dev)
            torch.ops.inferd.kv_advance(table, [0, 1, 2], 1)
            rg.launch()
            torch.cuda.synchronize()
            assert torch.equal(cur.cpu(), ref_ids.cpu())
        assert n == words.numel()
        torch.ops.inferd.graph_destroy(gr)
        assert torch.ops.inferd.kv_query(table, 0) == (44, 1)
    finally:
        torch.ops.inferd.kv_destroy(table)
        torch.ops.inferd.span_destroy(span)
