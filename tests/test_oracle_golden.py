"""Pin the CPU oracle (oracle/qwen3_ref.py) to golden vectors produced by the
reference's own modules (tests/golden/make_golden.py)."""
import torch

from golden_io import load, tensor
from oracle import qwen3_ref as R

SEED = 1234


def _maxabs(a, b):
    return (a.float() - b.float()).abs().max().item()


def test_units_rmsnorm_rope_qkrope_mlp():
    u = load("units.npz")
    d = R.CONFIGS["qwen3-0.6b"]
    w = R.gen_layer_weights(d, SEED, 0)["input_layernorm"]
    for tag, dt in (("bf16", torch.bfloat16), ("fp32", torch.float32)):
        x = tensor(u[f"rms_{tag}_x"])
        y = R.rms_norm(x, w.to(dt), d.eps)
        assert torch.equal(y, tensor(u[f"rms_{tag}_y"])), tag
        c, s = R.rope_cos_sin(d, torch.from_numpy(u["rope_pos"]), dt)
        assert torch.equal(c, tensor(u[f"rope_{tag}_cos"]))
        assert torch.equal(s, tensor(u[f"rope_{tag}_sin"]))
    W = R.gen_layer_weights(d, SEED, 3)
    q, k = tensor(u["qkr_q"]), tensor(u["qkr_k"])
    pos = torch.from_numpy(u["qkr_pos"])
    c, s = R.rope_cos_sin(d, pos, torch.bfloat16)
    qn = R.rms_norm(q, W["q_norm"], d.eps).transpose(1, 2)
    kn = R.rms_norm(k, W["k_norm"], d.eps).transpose(1, 2)
    qe, ke = R.apply_rope(qn, kn, c, s)
    assert torch.equal(qe, tensor(u["qkr_q_out"]))
    assert torch.equal(ke, tensor(u["qkr_k_out"]))
    y = R.mlp(tensor(u["mlp_x"]), W)
    assert torch.equal(y, tensor(u["mlp_y"]))


def test_tiny_petals_span_chain():
    g = load("tiny_petals.npz")
    d = R.CONFIGS["tiny"]
    prompt = torch.from_numpy(g["prompt"])[None]
    # fp32: the real PartitionedQwen2.forward chain (2 spans)
    s0 = R.RefSpan(d, SEED, 0, 1, True, False, torch.float32, "sdpa")
    s1 = R.RefSpan(d, SEED, 2, 3, False, True, torch.float32, "sdpa")
    h0 = s0.forward(prompt)
    assert _maxabs(h0, tensor(g["fp32_span0_hidden"])) < 1e-5
    lg = s1.forward(h0)
    assert _maxabs(lg, tensor(g["fp32_logits"])) < 1e-5
    ids = prompt[0].tolist()
    for _ in range(8):
        x = torch.tensor([ids])
        ids.append(R.greedy_token(s1.forward(s0.forward(x))))
    assert ids[16:] == g["fp32_greedy_ids"].tolist()
    # bf16 stage modules, per layer
    b0 = R.RefSpan(d, SEED, 0, 1, True, False, torch.bfloat16, "sdpa")
    b1 = R.RefSpan(d, SEED, 2, 3, False, True, torch.bfloat16, "sdpa")
    per = []
    h0 = b0.forward(prompt, per_layer=per)
    lg = b1.forward(h0, per_layer=per)
    for i, p in enumerate(per):
        assert torch.equal(p, tensor(g[f"bf16_layer{i}"])), i
    assert torch.equal(lg, tensor(g["bf16_logits"]))
    ids = prompt[0].tolist()
    for _ in range(8):
        ids.append(R.greedy_token(b1.forward(b0.forward(torch.tensor([ids])))))
    assert ids[16:] == g["bf16_greedy_ids"].tolist()
    one = R.RefSpan(d, SEED, 0, 3, True, True, torch.float32, "sdpa")
    assert _maxabs(one.forward(prompt), tensor(g["fp32_onespan_logits"])) < 1e-5


def _check_server(name, cfg, tags):
    g = load(name)
    d = R.CONFIGS[cfg]
    s, e = int(g["start"]), int(g["end"])
    for tag, dt, tol in tags:
        sp = R.RefSpan(d, SEED, s, e, False, False, dt, "eager")
        ndec = sum(1 for k in g.files if k.startswith(f"{tag}_in_dec"))
        outs = [sp.forward_cached("s", tensor(g[f"{tag}_in_prefill"]))]
        for i in range(ndec):
            outs.append(sp.forward_cached("s", tensor(g[f"{tag}_in_dec{i}"])))
        for i, o in enumerate(outs):
            ref = tensor(g[f"{tag}_out{i}"])
            if tol == 0:
                assert torch.equal(o, ref), (name, tag, i, _maxabs(o, ref))
            else:
                assert _maxabs(o, ref) <= tol, (name, tag, i, _maxabs(o, ref))


def test_tiny_server_cached():
    _check_server("tiny_server.npz", "tiny", (("fp32", torch.float32, 1e-5), ("bf16", torch.bfloat16, 0)))


def test_q06_layer_cached():
    _check_server("q06_layer.npz", "qwen3-0.6b", (("fp32", torch.float32, 1e-5), ("bf16", torch.bfloat16, 0)))


def test_q8b_layer_cached():
    _check_server("q8b_layer.npz", "qwen3-8b", (("bf16", torch.bfloat16, 0),))


def test_half_layer_spans_chain_equals_whole_layers():
    """The oracle's sub-layer stage boundaries (RefSpan skip_first_attn / skip_last_mlp, the
    engine's InferdSpanConfig flags) compose to the whole-layer span bit-exactly: the tiny model
    cut as [0..1a] [1m..2a] [2m..3] against one span, full recompute and cached prefill + 3 decode
    steps (the hand-off between halves is the bf16 residual h1 both compute); and the whole-layer
    span is still pinned to the reference-generated golden logits."""
    d = R.CONFIGS["tiny"]
    g = load("tiny_petals.npz")
    prompt = torch.from_numpy(g["prompt"])[None]
    cuts = [(0, 1, True, False, False, True), (1, 2, False, False, True, True), (2, 3, False, True, True, False)]
    chain = [R.RefSpan(d, SEED, a, b, f, l, torch.bfloat16, "sdpa", skip_first_attn=sf, skip_last_mlp=sl)
             for a, b, f, l, sf, sl in cuts]
    one = R.RefSpan(d, SEED, 0, d.layers - 1, True, True, torch.bfloat16, "sdpa")
    x = prompt
    for sp in chain:
        x = sp.forward(x)
    assert torch.equal(x, one.forward(prompt))
    assert torch.equal(x, tensor(g["bf16_logits"]))
    ids = prompt
    for step in range(4):
        x = ids
        for sp in chain:
            x = sp.forward_cached("s", x)
        y = one.forward_cached("s", ids)
        assert torch.equal(x, y), step
        ids = torch.argmax(y[:, -1], -1)[:, None]


def test_sublayer_record_spans_chain_equals_whole_layers():
    """The oracle's attention|o and q/k/v|attention boundaries (RefSpan o_split_* / qkv_split_*):
    the tiny model cut as [0..1 before o] [1 o.. 2 after q/k/v] [2 attention..3] composes to the
    whole-layer span bit-exactly -- the hand-offs are the records (x, attention output) and
    (x, raw q/k/v rows), or x alone where a q/k/v cut's call is not a pure decode call -- full
    recompute and cached prefill + 3 decode steps, pinned to the reference-generated golden logits."""
    d = R.CONFIGS["tiny"]
    g = load("tiny_petals.npz")
    prompt = torch.from_numpy(g["prompt"])[None]
    chain = [R.RefSpan(d, SEED, 0, 1, True, False, torch.bfloat16, "sdpa", o_split_last=True),
             R.RefSpan(d, SEED, 1, 2, False, False, torch.bfloat16, "sdpa", o_split_first=True, qkv_split_last=True),
             R.RefSpan(d, SEED, 2, 3, False, True, torch.bfloat16, "sdpa", qkv_split_first=True)]
    one = R.RefSpan(d, SEED, 0, d.layers - 1, True, True, torch.bfloat16, "sdpa")

    def run(fwd, x, decode):
        x = fwd(chain[0], x)                        # (x, attention output)
        xq = fwd(chain[1], x)                       # (x, q/k/v rows)
        return fwd(chain[2], xq if decode else (xq[0], None))

    x = run(lambda sp, v: sp.forward(v), prompt, False)
    assert torch.equal(x, one.forward(prompt))
    assert torch.equal(x, tensor(g["bf16_logits"]))
    ids = prompt
    for step in range(4):
        x = run(lambda sp, v: sp.forward_cached("s", v), ids, step > 0)
        y = one.forward_cached("s", ids)
        assert torch.equal(x, y), step
        ids = torch.argmax(y[:, -1], -1)[:, None]
