"""The vocab-parallel greedy head (ABI 5: InferdSpanConfig head_first / head_rows / final_norm_out,
inferd_span_head_shard, inferd_argmax_combine) against the whole head, bit for bit.

The reference's last span takes argmax(lm_head(norm(x))[:, -1]) (partitioned_models.py:95-96,162)
over the whole vocabulary on one stage.  Split over stages, each shard's GEMV computes its logits
with the same 16-column tiles over the whole K range, so every logit -- and therefore the max key
(order(logit) << 32 | ~global index) and its lowest-index tie-break -- is the one a single lm_head
computes: the tests below assert torch.equal on logits and ids, no tolerance."""
import pytest
import torch

from oracle import qwen3_ref as R

pytestmark = pytest.mark.gpu

SEED = 1234
DEV = "cuda"


def _span(cfg, first, n, profile="random", **kw):
    from inferd_amd.runtime import MODELS, SpanRuntime
    s = SpanRuntime(MODELS[cfg], first, n, device=DEV, max_positions=512, max_tokens=kw.pop("max_tokens", 1024),
                    max_seqs=kw.pop("max_seqs", 16), kv_pages=kw.pop("kv_pages", 64), **kw)
    s.init_synthetic(SEED, profile)
    return s


SHARDS_Q06 = [(0, 37888), (37888, 16), (37904, 60000), (97904, 54032)]   # uneven, one of a single tile


@pytest.mark.parametrize("cfg,B", [("qwen3-0.6b", 5), ("qwen3-8b", 16)])
def test_head_shards_chain_equals_whole_head(cfg, B):
    """The last layer of the model as (a) a span with the whole head and (b) a final_norm_out span
    whose normed rows go through lm_head shards chained by running keys: the ids are identical, the
    shards' logits concatenated are the whole head's logits bit for bit, and the keys combined at
    once (inferd_argmax_combine) give the same ids -- for a prefill call and two decode steps."""
    from inferd_amd.runtime import MODELS
    d = MODELS[cfg]
    V = d.vocab
    shards = SHARDS_Q06 if cfg == "qwen3-0.6b" else [(0, 18944), (18944, 18944), (37888, 56960), (94848, 57088)]
    assert sum(n for _, n in shards) == V
    L = d.layers - 1
    whole = _span(cfg, L, 1, has_embed=False, has_lm_head=True)
    tail = _span(cfg, L, 1, has_embed=False, has_lm_head=False, final_norm_out=True)
    heads = [_span(cfg, 0, 0, has_embed=False, has_lm_head=False, head_first=f, head_rows=n) for f, n in shards]
    g = torch.Generator().manual_seed(5)
    T = 9
    sess = [f"s{b}" for b in range(B)]
    x = (torch.randn(B * T, d.hidden, generator=g) * 0.7).to(torch.bfloat16)
    calls = [([(sid, T) for sid in sess], x)] + \
            [([(sid, 1) for sid in sess], (torch.randn(B, d.hidden, generator=g) * 0.7).to(torch.bfloat16))
             for _ in range(2)]
    for reqs, xc in calls:
        ow = whole.forward(reqs, x=xc, want_hidden=False, want_next_ids=True, want_logits=True)
        nt = tail.forward(reqs, x=xc)["hidden"]
        assert nt.numel() == (B + 15) // 16 * 16 * d.hidden
        keys = None
        all_keys = torch.zeros(len(shards), B, dtype=torch.int64, device=DEV)
        parts = []
        ids = torch.empty(B, dtype=torch.int32, device=DEV)
        for i, (sp, (f, n)) in enumerate(zip(heads, shards)):
            lg = torch.empty(B, n, dtype=torch.bfloat16, device=DEV)
            ko = torch.empty(B, dtype=torch.int64, device=DEV)
            sp.head_shard(nt, B, keys_in=keys, keys_out=ko, ids=ids if i == len(shards) - 1 else None, logits=lg)
            sp.head_shard(nt, B, keys_out=all_keys[i])
            keys = ko
            parts.append(lg)
        torch.cuda.synchronize()
        assert torch.equal(torch.cat(parts, 1), ow["logits"])
        assert torch.equal(ids, ow["next_ids"]), (ids, ow["next_ids"])
        ids2 = torch.empty(B, dtype=torch.int32, device=DEV)
        torch.ops.inferd.argmax_combine(all_keys, len(shards), B, ids2)
        assert torch.equal(ids2, ow["next_ids"])
        # the whole-head span reduces all rows through the same entry point
        ids3 = torch.empty(B, dtype=torch.int32, device=DEV)
        whole.head_shard(nt, B, ids=ids3)     # the same normed rows (the same final norm weight)
        torch.cuda.synchronize()
        assert torch.equal(ids3, ow["next_ids"])
        ref = torch.argmax(ow["logits"].float().cpu(), -1).to(torch.int32)
        assert torch.equal(ids.cpu(), ref)


def test_head_shard_ties_go_to_the_lowest_index():
    """Rows a < b in different shards set to the same vector, large against sequence 0's normed row:
    both logits are equal and maximal; the chained shards (in either order) and the combine pick a,
    as torch.argmax does."""
    from inferd_amd.runtime import MODELS, GLOBAL_TENSOR_IDS, gen_tensor
    cfg = "qwen3-0.6b"
    d = MODELS[cfg]
    shards = SHARDS_Q06
    a, b = 5000, 120008      # the same column within their 16-column tiles
    tail = _span(cfg, d.layers - 1, 1, has_embed=False, has_lm_head=False, final_norm_out=True)
    heads = [_span(cfg, 0, 0, has_embed=False, has_lm_head=False, head_first=f, head_rows=n) for f, n in shards]
    B = 3
    x = (torch.randn(B, d.hidden, generator=torch.Generator().manual_seed(8)) * 0.7).to(torch.bfloat16)
    nt = tail.forward([(None, 1)] * B, x=x)["hidden"]
    from inferd_amd.pipeline import unpack_rows
    v = (unpack_rows(nt, B, d.hidden)[0].float() * 4).to(torch.bfloat16)
    lm = gen_tensor(SEED, GLOBAL_TENSOR_IDS["lm_head"], (d.vocab, d.hidden), False, DEV)
    lm[a] = v
    lm[b] = v
    for sp, (f, n) in zip(heads, shards):
        sp.set_weight(-1, "lm_head", lm[f:f + n].contiguous())
    for order in (range(len(shards)), reversed(range(len(shards)))):
        keys, ids = None, torch.empty(B, dtype=torch.int32, device=DEV)
        order = list(order)
        for j, i in enumerate(order):
            ko = torch.empty(B, dtype=torch.int64, device=DEV)
            heads[i].head_shard(nt, B, keys_in=keys, keys_out=ko, ids=ids if j == len(order) - 1 else None)
            keys = ko
        torch.cuda.synchronize()
        assert int(ids[0]) == a, (order, ids)
    # and torch.argmax over the same bf16 logits agrees
    lg = torch.nn.functional.linear(unpack_rows(nt, B, d.hidden)[:1].float(), lm.float())
    assert int(torch.argmax(lg)) == a


def test_final_norm_out_decode_graph_and_oracle():
    """A final_norm_out span stepped as a decode graph writes the same normed rows as its eager
    forward, and they are within the span tolerance of the oracle's final norm (RefSpan with
    final_norm_out)."""
    from inferd_amd.pipeline import unpack_rows
    from inferd_amd.runtime import MODELS, DecodeGraph
    cfg = "qwen3-0.6b"
    d = MODELS[cfg]
    B, T = 4, 12
    g = torch.Generator().manual_seed(3)
    x = (torch.randn(B * T, d.hidden, generator=g) * 0.7).to(torch.bfloat16)
    steps = (torch.randn(3, B, d.hidden, generator=g) * 0.7).to(torch.bfloat16)
    outs = []
    for graph in (False, True):
        sp = _span(cfg, d.layers - 2, 2, has_embed=False, has_lm_head=False, final_norm_out=True)
        sess = [f"n{b}" for b in range(B)]
        sp.forward([(s, T) for s in sess], x=x, want_hidden=False)
        xin = torch.zeros(B, d.hidden, dtype=torch.bfloat16, device=DEV)
        nout = torch.zeros(sp.normed_elems(B), dtype=torch.bfloat16, device=DEV)
        gr = DecodeGraph(sp, sess, 3, x=xin, hidden_out=nout) if graph else None
        seq = []
        for k in range(3):
            xin.copy_(steps[k])
            if graph:
                gr.launch_eager() if k == 1 else gr.launch()
                seq.append(nout.clone())
            else:
                seq.append(sp.forward([(s, 1) for s in sess], x=xin)["hidden"].clone())
        outs.append(torch.stack(seq))
    assert torch.equal(outs[0], outs[1])
    ref = R.RefSpan(R.CONFIGS[cfg], SEED, d.layers - 2, d.layers - 1, False, False, final_norm_out=True)
    ref.forward_cached("o", x.view(B, T, -1)[:1])
    want = ref.forward_cached("o", steps[0][:1, None])[0, 0]
    got = unpack_rows(outs[0][0], B, d.hidden)[0]
    e = ((got.float().cpu() - want.float()).abs().max() / want.float().abs().max()).item()
    print(f"final_norm_out vs oracle: max_norm {e:.2e}")
    assert e < 2e-2


def test_head_configs_refused():
    from inferd_amd.runtime import MODELS, SpanRuntime
    d = MODELS["tiny"]
    bad = [dict(has_lm_head=True, head_rows=16), dict(has_lm_head=True, final_norm_out=True),
           dict(head_first=8, head_rows=16), dict(head_first=1024, head_rows=16), dict(head_rows=24),
           dict(final_norm_out=True, skip_last_mlp=True)]
    for kw in bad:
        kw = {"has_lm_head": False, **kw}
        with pytest.raises(RuntimeError):
            SpanRuntime(d, 0, 2, has_embed=False, device=DEV, **kw)
    sp = SpanRuntime(d, 0, 2, has_embed=False, has_lm_head=False, device=DEV)
    with pytest.raises(RuntimeError):     # no rows to reduce
        sp.head_shard(torch.zeros(16 * d.hidden, dtype=torch.bfloat16, device=DEV), 2,
                      keys_out=torch.zeros(2, dtype=torch.int64, device=DEV))
