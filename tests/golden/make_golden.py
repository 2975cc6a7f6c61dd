"""Generate the golden vectors under tests/golden/ by running the REFERENCE's own code.

Run in the build container only (needs /root/reference; never runs on the GPU box):
    python tests/golden/make_golden.py

What it drives (all on CPU, synthetic weights from oracle/weightgen.py, no network):
  * petals span path: `petals/partitioned_models.py` -- the real `PartitionedQwen2.forward`
    (object created with __new__ so no checkpoint/tokenizer fetch; the pickled
    `torch.load` at :112-116 is replaced by attribute injection of the same
    First/Last stage modules built from HF `Qwen3DecoderLayer`, attn 'sdpa') and the
    stage modules `FirstStage`/`StageInner`/`LastStage` directly (bf16: the codec at
    :11-26 cannot carry bf16).  HF 5.x layers return a Tensor, so each layer is
    wrapped to restore the 4.52.4 `(hidden,)` tuple contract.
  * gRPC span path: `models/qwen3/server/qwen3_server_module.py` -- `Qwen3Server.send`
    with a per-session DynamicCache (`_load_weights` overridden: no hub download),
    prefill then single-token cached decode with the masks of client.py:221-224/249-250.
  * unit vectors: Qwen3RMSNorm, rotary tables, QK-norm + RoPE, SwiGLU MLP.

Outputs are small .npz files (bf16 payloads stored as uint16 bit patterns).
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np
import torch
from torch import nn

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REF = "/root/reference"
OUT = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REF, "models", "qwen3"))
sys.path.insert(0, os.path.join(REF, "models", "qwen3", "server"))
sys.path.insert(0, os.path.join(REF, "petals"))

from oracle import qwen3_ref as R  # noqa: E402  (weights + dims only)

import qwen3_config  # noqa: E402
import qwen3_server_module as QS  # noqa: E402
import partitioned_models as PM  # noqa: E402
from transformers import Qwen3Config as HFQwen3Config  # noqa: E402
from transformers.models.qwen3 import modeling_qwen3 as HFQ  # noqa: E402

SEED = 1234
torch.manual_seed(0)


def bits(t: torch.Tensor) -> np.ndarray:
    return t.detach().to(torch.bfloat16).contiguous().view(torch.int16).numpy().view(np.uint16).copy()


def f32(t: torch.Tensor) -> np.ndarray:
    return t.detach().to(torch.float32).numpy().copy()


def out_of(t: torch.Tensor) -> np.ndarray:
    return bits(t) if t.dtype == torch.bfloat16 else f32(t)


# ----------------------------------------------------------------------------- helpers
def set_ref_config(d: R.Qwen3Dims):
    C = qwen3_config.Qwen3Config
    C.HIDDEN_SIZE, C.INTERMEDIATE_SIZE = d.hidden, d.intermediate
    C.NUM_ATTENTION_HEADS, C.NUM_KEY_VALUE_HEADS = d.heads, d.kv_heads
    C.NUM_HIDDEN_LAYERS, C.VOCAB_SIZE, C.HEAD_DIM = d.layers, d.vocab, d.head_dim


def layer_state_dict(W: dict) -> dict:
    sd = {}
    for n in ("q_proj", "k_proj", "v_proj", "o_proj", "q_norm", "k_norm"):
        sd[f"self_attn.{n}.weight"] = W[n]
    for n in ("gate_proj", "up_proj", "down_proj"):
        sd[f"mlp.{n}.weight"] = W[n]
    sd["input_layernorm.weight"] = W["input_layernorm"]
    sd["post_attention_layernorm.weight"] = W["post_attention_layernorm"]
    return sd


def hf_config(d: R.Qwen3Dims) -> HFQwen3Config:
    return HFQwen3Config(hidden_size=d.hidden, intermediate_size=d.intermediate,
                         num_attention_heads=d.heads, num_key_value_heads=d.kv_heads,
                         head_dim=d.head_dim, num_hidden_layers=d.layers, vocab_size=d.vocab,
                         rope_theta=d.rope_theta, rms_norm_eps=d.eps, attention_bias=False,
                         max_position_embeddings=d.max_positions, attn_implementation="sdpa")


class TupleShim(nn.Module):
    """Restore the transformers-4.52.4 decoder-layer contract `layer(...)[0]`."""

    def __init__(self, layer):
        super().__init__()
        self.layer = layer

    def forward(self, *a, **k):
        out = self.layer(*a, **k)
        return out if isinstance(out, tuple) else (out,)


def build_petals_stages(d, spans, dtype, profile="random"):
    """spans: list of (start, end).  Returns the reference stage modules."""
    cfg = hf_config(d)
    g = R.gen_global_weights(d, SEED, dtype, profile)
    embed = nn.Embedding(d.vocab, d.hidden).to(dtype)
    embed.weight.data.copy_(g["embed_tokens"])
    norm = HFQ.Qwen3RMSNorm(d.hidden, eps=d.eps).to(dtype)
    norm.weight.data.copy_(g["norm"])
    lm_head = nn.Linear(d.hidden, d.vocab, bias=False).to(dtype)
    lm_head.weight.data.copy_(g["lm_head"])
    rotary = HFQ.Qwen3RotaryEmbedding(cfg)
    mods = []
    for si, (s, e) in enumerate(spans):
        layers = []
        for i in range(s, e + 1):
            L = HFQ.Qwen3DecoderLayer(cfg, i).to(dtype)
            L.load_state_dict(layer_state_dict(R.gen_layer_weights(d, SEED, i, dtype)))
            layers.append(TupleShim(L))
        if si == 0 and len(spans) == 1:
            # one span that is both first and last: FirstStage then final norm/lm_head
            m = PM.FirstStage(embed, rotary, layers)
            m.norm, m.lm_head = norm, lm_head
        elif si == 0:
            m = PM.FirstStage(embed, rotary, layers)
        elif si == len(spans) - 1:
            m = PM.LastStage(rotary, layers, norm, lm_head)
        else:
            m = PM.StageInner(rotary, layers)
        mods.append(m.eval())
    return mods


class _TokStub:
    def decode(self, i):
        return f"<{i}>"


def partitioned(stage, num_stages, module):
    """A real PartitionedQwen2 without the checkpoint/tokenizer fetch of :103-117."""
    p = object.__new__(PM.PartitionedQwen2)
    p.stage, p.num_stages, p.parts_path = stage, num_stages, "<injected>"
    p.device = torch.device("cpu")
    p.tokenizer = _TokStub()
    p.model = module
    return p


# ----------------------------------------------------------------------------- fixtures
def gen_tiny_petals():
    d = R.CONFIGS["tiny"]
    rng = np.random.default_rng(7)
    prompt = rng.integers(0, d.vocab, size=16).tolist()
    res = {"prompt": np.array(prompt, dtype=np.int64)}
    # (1) real PartitionedQwen2.forward chain, fp32, 2 spans [0-1],[2-3]: greedy 8 tokens
    s0, s1 = build_petals_stages(d, [(0, 1), (2, 3)], torch.float32)
    n0, n1 = partitioned(0, 2, s0), partitioned(1, 2, s1)
    ids = list(prompt)
    first_hidden = None
    for step in range(8):
        o0 = n0.forward({"generated_ids": ids})
        if first_hidden is None:
            first_hidden = PM.base64_to_tensor(o0["hidden_meta"])
        o1 = n1.forward(o0)
        ids = o1["generated_ids"]
    res["fp32_span0_hidden"] = f32(first_hidden)
    res["fp32_greedy_ids"] = np.array(ids[len(prompt):], dtype=np.int64)
    with torch.no_grad():
        att = torch.ones((1, 16), dtype=torch.long)
        mask = PM.build_decoder_attention_mask(att)
        pos = torch.arange(16).unsqueeze(0)
        res["fp32_logits"] = f32(s1(first_hidden, mask, pos))
    # (2) bf16 stage modules directly (codec cannot carry bf16), per-layer capture
    for dt, tag in ((torch.bfloat16, "bf16"),):
        s0, s1 = build_petals_stages(d, [(0, 1), (2, 3)], dt)
        caps = []
        for st in (s0, s1):
            for m in st.layers:
                m.layer.register_forward_hook(lambda mod, a, o: caps.append(o if torch.is_tensor(o) else o[0]))
        with torch.no_grad():
            x = torch.tensor([prompt])
            att = torch.ones((1, 16), dtype=torch.long)
            mask = PM.build_decoder_attention_mask(att)
            pos = torch.arange(16).unsqueeze(0)
            h0 = s0(x, mask, pos)
            lg = s1(h0, mask, pos)
        res[f"{tag}_span0_hidden"] = out_of(h0)
        res[f"{tag}_logits"] = out_of(lg)
        for i, c in enumerate(caps):
            res[f"{tag}_layer{i}"] = out_of(c)
        # greedy loop, full recompute (send_message.py:46-60 semantics)
        ids = list(prompt)
        for step in range(8):
            with torch.no_grad():
                T = len(ids)
                m = PM.build_decoder_attention_mask(torch.ones((1, T), dtype=torch.long))
                p = torch.arange(T).unsqueeze(0)
                lg = s1(s0(torch.tensor([ids]), m, p), m, p)
            ids.append(int(torch.argmax(lg[:, -1, :], dim=-1).item()))
        res[f"{tag}_greedy_ids"] = np.array(ids[len(prompt):], dtype=np.int64)
    # (3) one span holding all 4 layers (first+last) in fp32
    (s,) = build_petals_stages(d, [(0, 3)], torch.float32)
    with torch.no_grad():
        x = torch.tensor([prompt])
        mask = PM.build_decoder_attention_mask(torch.ones((1, 16), dtype=torch.long))
        pos = torch.arange(16).unsqueeze(0)
        h = s(x, mask, pos)
        res["fp32_onespan_logits"] = f32(s.lm_head(s.norm(h)))
    np.savez_compressed(os.path.join(OUT, "tiny_petals.npz"), **res)


def gen_tiny_petals_peaked(steps=16):
    """The tiny model with the peaked embed / lm_head profile (oracle/weightgen.py): large top-1
    margins, so a GPU chain must reproduce EVERY id of the reference's own chain.  (1) the real
    PartitionedQwen2.forward chain (fp32 codec), (2) the bf16 stage modules, both free-running
    greedy with full recompute (send_message.py:46-60) for `steps` steps; the bf16 top-2 margins
    are recorded."""
    d = R.CONFIGS["tiny"]
    rng = np.random.default_rng(17)
    prompt = rng.integers(0, d.vocab, size=16).tolist()
    res = {"prompt": np.array(prompt, dtype=np.int64)}
    s0, s1 = build_petals_stages(d, [(0, 1), (2, 3)], torch.float32, "peaked")
    n0, n1 = partitioned(0, 2, s0), partitioned(1, 2, s1)
    ids = list(prompt)
    for step in range(steps):
        ids = n1.forward(n0.forward({"generated_ids": ids}))["generated_ids"]
    res["fp32_greedy_ids"] = np.array(ids[len(prompt):], dtype=np.int64)
    s0, s1 = build_petals_stages(d, [(0, 1), (2, 3)], torch.bfloat16, "peaked")
    ids, margins = list(prompt), []
    for step in range(steps):
        with torch.no_grad():
            T = len(ids)
            m = PM.build_decoder_attention_mask(torch.ones((1, T), dtype=torch.long))
            p = torch.arange(T).unsqueeze(0)
            lg = s1(s0(torch.tensor([ids]), m, p), m, p)[0, -1]
        top = torch.topk(lg.float(), 2).values
        margins.append(float(top[0] - top[1]))
        ids.append(int(torch.argmax(lg).item()))
    res["bf16_greedy_ids"] = np.array(ids[len(prompt):], dtype=np.int64)
    res["bf16_margins"] = np.array(margins, dtype=np.float32)
    np.savez_compressed(os.path.join(OUT, "tiny_petals_peaked.npz"), **res)
    print("tiny_petals_peaked: fp32", res["fp32_greedy_ids"].tolist(), "bf16", res["bf16_greedy_ids"].tolist(),
          "min margin", min(margins))


class _Server(QS.Qwen3Server):
    def _load_weights(self):  # no hub download: weights injected below
        pass


def run_server(d, start, end, dtype, hidden_prefill, decode_hiddens, sid="s0"):
    set_ref_config(d)
    srv = _Server(start, end).to(dtype)
    for L in srv.local_layers:
        L.load_state_dict(layer_state_dict(R.gen_layer_weights(d, SEED, L.self_attn.layer_idx, dtype)))
    cfg = hf_config(d)
    rot = HFQ.Qwen3RotaryEmbedding(cfg)
    outs = []
    with torch.no_grad():
        B, T, _ = hidden_prefill.shape
        pos = torch.arange(T).unsqueeze(0).expand(B, T)
        min_val = torch.finfo(dtype).min
        tril = torch.tril(torch.ones(T, T, dtype=dtype))
        mask = ((1.0 - tril) * min_val).unsqueeze(0).unsqueeze(0).expand(B, 1, T, T)   # client.py:221-224
        cos, sin = rot(hidden_prefill, pos)
        outs.append(srv.send(sid, hidden_prefill, mask, pos[0], (cos, sin)))
        for i, h in enumerate(decode_hiddens):
            p = torch.full((B, 1), T + i)
            m1 = torch.zeros((1, 1), dtype=dtype).unsqueeze(0).unsqueeze(0)           # client.py:249-250
            cos, sin = rot(h, p)
            outs.append(srv.send(sid, h, m1, p[0], (cos, sin)))
    return outs


def gen_server(name, cfgname, start, end, B, T, ndec, dtypes, seed):
    d = R.CONFIGS[cfgname]
    g = torch.Generator().manual_seed(seed)
    hp = torch.randn((B, T, d.hidden), generator=g)
    hd = [torch.randn((B, 1, d.hidden), generator=g) for _ in range(ndec)]
    res = {"start": np.int64(start), "end": np.int64(end)}
    for dt, tag in dtypes:
        hp_d = hp.to(dt)
        hd_d = [x.to(dt) for x in hd]
        res[f"{tag}_in_prefill"] = out_of(hp_d)
        for i, x in enumerate(hd_d):
            res[f"{tag}_in_dec{i}"] = out_of(x)
        outs = run_server(d, start, end, dt, hp_d, hd_d)
        for i, o in enumerate(outs):
            res[f"{tag}_out{i}"] = out_of(o)
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **res)


def gen_units():
    d = R.CONFIGS["qwen3-0.6b"]
    set_ref_config(d)
    g = torch.Generator().manual_seed(11)
    res = {}
    # RMSNorm (qwen3_server_module.py:14-25) in bf16 and fp32
    x = torch.randn((8, d.hidden), generator=g) * 3.0
    w = R.gen_layer_weights(d, SEED, 0, torch.bfloat16)["input_layernorm"]
    for dt, tag in ((torch.bfloat16, "bf16"), (torch.float32, "fp32")):
        n = QS.Qwen3RMSNorm(d.hidden, eps=d.eps).to(dt)
        n.weight.data.copy_(w.to(dt))
        res[f"rms_{tag}_x"] = out_of(x.to(dt))
        res[f"rms_{tag}_y"] = out_of(n(x.to(dt)).detach())
    # rotary tables at assorted positions (HF Qwen3RotaryEmbedding, the petals `rotary`)
    rot = HFQ.Qwen3RotaryEmbedding(hf_config(d))
    pos = torch.tensor([[0, 1, 2, 3, 17, 255, 1000, 2047, 2048, 4095, 8191, 12345, 32767, 40959]])
    for dt, tag in ((torch.bfloat16, "bf16"), (torch.float32, "fp32")):
        c, s = rot(torch.zeros(1, dtype=dt), pos)
        res["rope_pos"] = pos.numpy()
        res[f"rope_{tag}_cos"] = out_of(c)
        res[f"rope_{tag}_sin"] = out_of(s)
    # QK-norm + RoPE (qwen3_server_module.py:134-142) on one token block, bf16
    W = R.gen_layer_weights(d, SEED, 3, torch.bfloat16)
    att = QS.Qwen3Attention(3).to(torch.bfloat16)
    att.q_norm.weight.data.copy_(W["q_norm"])
    att.k_norm.weight.data.copy_(W["k_norm"])
    T = 6
    q = (torch.randn((1, T, d.heads, d.head_dim), generator=g) * 2).to(torch.bfloat16)
    k = (torch.randn((1, T, d.kv_heads, d.head_dim), generator=g) * 2).to(torch.bfloat16)
    p = torch.arange(100, 100 + T).unsqueeze(0)
    c, s = rot(q, p)
    qn = att.q_norm(q).transpose(1, 2)
    kn = att.k_norm(k).transpose(1, 2)
    qe, ke = QS.apply_rotary_pos_emb(qn, kn, c, s)
    res.update(qkr_q=bits(q), qkr_k=bits(k), qkr_pos=p.numpy(), qkr_q_out=bits(qe), qkr_k_out=bits(ke))
    # SwiGLU MLP (qwen3_server_module.py:28-40), bf16
    mlp = QS.Qwen3MLP().to(torch.bfloat16)
    for n in ("gate_proj", "up_proj", "down_proj"):
        getattr(mlp, n).weight.data.copy_(W[n])
    xm = (torch.randn((4, d.hidden), generator=g)).to(torch.bfloat16)
    res.update(mlp_x=bits(xm), mlp_y=bits(mlp(xm).detach()))
    np.savez_compressed(os.path.join(OUT, "units.npz"), **res)


def gen_codec():
    """The reference's wire codec and mask builder on fixed inputs (partitioned_models.py:11-35)."""
    import json
    t = (torch.arange(24, dtype=torch.float32).reshape(1, 4, 6) - 7.5) / 3.0
    meta = PM.tensor_to_base64(t)
    mask = PM.build_decoder_attention_mask(torch.tensor([[1, 1, 1, 0, 1]]))
    with open(os.path.join(OUT, "codec.json"), "w") as f:
        json.dump({"input": t.reshape(-1).tolist(), "shape": list(t.shape), "meta": meta,
                   "mask": mask.to(torch.int32).reshape(-1).tolist(), "mask_shape": list(mask.shape)}, f)


if __name__ == "__main__":
    os.makedirs(OUT, exist_ok=True)
    if len(sys.argv) > 1:   # named generators only, e.g. `make_golden.py tiny_petals_peaked`
        for name in sys.argv[1:]:
            globals()[f"gen_{name}"]()
        sys.exit(0)
    gen_codec()
    gen_units()
    gen_tiny_petals()
    gen_tiny_petals_peaked()
    gen_server("tiny_server", "tiny", 0, 3, 1, 8, 4, ((torch.float32, "fp32"), (torch.bfloat16, "bf16")), 21)
    gen_server("q06_layer", "qwen3-0.6b", 5, 5, 1, 8, 4, ((torch.float32, "fp32"), (torch.bfloat16, "bf16")), 22)
    gen_server("q8b_layer", "qwen3-8b", 7, 7, 2, 4, 2, ((torch.bfloat16, "bf16"),), 23)
    for f in sorted(os.listdir(OUT)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(OUT, f)))
