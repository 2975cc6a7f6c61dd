"""Offline span builder: the equivalent of the reference's `split_model.py`.

Reads the reference's span config (`petals/inferd.yaml` format: model_name, parts_dir,
stages_count, stages[{name, stage, start_layer, end_layer}], split_model.py:76-79) and
writes one safetensors stage file per entry: `<parts_dir>/<name>/model.safetensors` with
the span's layer weights under `layers.<j>.<state-dict key>` (j span-local, keys as in
Qwen3DecoderLayer, qwen3_server_module.py:165-176), plus `embed.weight` (first stage) and
`norm.weight` / `lm_head.weight` (last stage), and the model dims + span range in the
file metadata.  PartitionedQwen2 loads these with safetensors (nothing executes on load),
instead of the reference's pickled `torch.save(module)` (split_model.py:107).

Roles come from the entry's `stage` field against `stages_count` -- so the reference's
quirk of building `node2` (stage 2 of 3) as a StageInner because the yaml lists four
entries (split_model.py:91-102) does not carry over.

Weight sources: a HF-format safetensors checkpoint directory (keys `model.layers.{i}.*`,
`model.embed_tokens.weight`, `model.norm.weight`, `lm_head.weight`, tied embeddings
allowed; the model geometry from its config.json, so any Qwen3 size loads; other
architectures -- the reference's default Qwen2-0.5B among them -- are refused with the reason)
or the counter-based synthetic generator (`--synthetic-seed`).
"""
from __future__ import annotations

import argparse
import json
import os
from dataclasses import asdict

import torch
import yaml

from .runtime import MODELS, ModelDims

LAYER_KEYS = ("self_attn.q_proj.weight", "self_attn.k_proj.weight", "self_attn.v_proj.weight",
              "self_attn.o_proj.weight", "self_attn.q_norm.weight", "self_attn.k_norm.weight",
              "mlp.gate_proj.weight", "mlp.up_proj.weight", "mlp.down_proj.weight",
              "input_layernorm.weight", "post_attention_layernorm.weight")


def write_stage_file(path: str, dims: ModelDims, start: int, end: int, first: bool, last: bool,
                     get_layer, get_global):
    """get_layer(i) -> {state-dict key: tensor} of global layer i; get_global(name) for
    'embed_tokens' / 'norm' / 'lm_head'."""
    from safetensors.torch import save_file
    tensors = {}
    for j, i in enumerate(range(start, end + 1)):
        for k, v in get_layer(i).items():
            tensors[f"layers.{j}.{k}"] = v.to(torch.bfloat16).contiguous()
    if first:
        tensors["embed.weight"] = get_global("embed_tokens").to(torch.bfloat16).contiguous()
    if last:
        tensors["norm.weight"] = get_global("norm").to(torch.bfloat16).contiguous()
        tensors["lm_head.weight"] = get_global("lm_head").to(torch.bfloat16).contiguous()
    meta = {"dims": json.dumps(asdict(dims)), "start_layer": str(start), "end_layer": str(end),
            "first": "1" if first else "0", "last": "1" if last else "0"}
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    save_file(tensors, path, metadata=meta)


def checkpoint_dims(ckpt_dir: str, name: str | None = None) -> ModelDims | None:
    """The model geometry of a HF checkpoint directory from its config.json (None without one),
    so any Qwen3 size loads (4B, 14B, ... -- not only the sizes in runtime.MODELS).  Anything
    but a Qwen3 decoder is refused here with the reason, instead of failing later on a missing
    key or a shape: the reference's petals config names Qwen/Qwen2-0.5B (petals/inferd.yaml:1,
    loaded by split_model.py:81 as Qwen2ForCausalLM), whose layers carry q/k/v biases, no
    QK-norm and 64-dim heads; this engine implements the Qwen3 layer (qwen3_server_module.py,
    BASELINE north_star).  Rotary scaling other than the default is refused too (the rope
    tables are the HF default formula, client.py:56-71)."""
    p = os.path.join(ckpt_dir, "config.json")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        c = json.load(f)
    mt = c.get("model_type", "")
    if mt != "qwen3":
        raise ValueError(f"{ckpt_dir}: model_type {mt!r} -- this engine runs Qwen3 decoder layers (QK-norm, "
                         "no q/k/v bias, 128-dim heads); a Qwen2 checkpoint (the reference's default "
                         "Qwen/Qwen2-0.5B) has biases, no QK-norm and 64-dim heads")
    hd = c.get("head_dim") or c["hidden_size"] // c["num_attention_heads"]
    if hd != 128:
        raise ValueError(f"{ckpt_dir}: head_dim {hd}; the engine's attention kernels take 128")
    if c.get("attention_bias"):
        raise ValueError(f"{ckpt_dir}: attention_bias is set; the engine's projections have no bias")
    if c.get("rope_scaling"):
        raise ValueError(f"{ckpt_dir}: rope_scaling {c['rope_scaling']!r}; the engine's rope tables are the "
                         "default (unscaled) formula")
    return ModelDims(name=name or os.path.basename(os.path.normpath(ckpt_dir)), hidden=c["hidden_size"],
                     intermediate=c["intermediate_size"], heads=c["num_attention_heads"],
                     kv_heads=c["num_key_value_heads"], layers=c["num_hidden_layers"], vocab=c["vocab_size"],
                     head_dim=hd, eps=float(c.get("rms_norm_eps", 1e-6)),
                     rope_theta=float(c.get("rope_theta", 1_000_000.0)),
                     max_positions=int(c.get("max_position_embeddings", 40960)))


def hf_checkpoint_source(ckpt_dir: str):
    """Lazy accessors over a HF safetensors checkpoint (sharded or single file).  Refuses biased
    projections (Qwen2-style layers) up front (checkpoint_dims)."""
    from safetensors import safe_open
    files = [os.path.join(ckpt_dir, f) for f in sorted(os.listdir(ckpt_dir)) if f.endswith(".safetensors")]
    where = {}
    for fn in files:
        with safe_open(fn, framework="pt", device="cpu") as f:
            for k in f.keys():
                where[k] = fn
    biased = sorted(k for k in where if k.endswith("_proj.bias"))
    if biased:
        raise ValueError(f"{ckpt_dir}: biased projections ({biased[0]}, ...) -- Qwen2-style layers, not a Qwen3 "
                         "checkpoint (checkpoint_dims)")

    def get(key):
        with safe_open(where[key], framework="pt", device="cpu") as f:
            return f.get_tensor(key)

    def get_layer(i):
        return {k: get(f"model.layers.{i}.{k}") for k in LAYER_KEYS}

    def get_global(name):
        if name == "lm_head" and "lm_head.weight" not in where:   # tie_word_embeddings
            return get("model.embed_tokens.weight")
        return get({"embed_tokens": "model.embed_tokens.weight", "norm": "model.norm.weight",
                    "lm_head": "lm_head.weight"}[name])
    return get_layer, get_global


def split(cfg: dict, dims: ModelDims, get_layer, get_global, out_dir: str | None = None) -> list:
    parts_dir = out_dir or cfg["parts_dir"]
    n_stages = int(cfg["stages_count"])
    written = []
    for st in cfg["stages"]:
        stage = int(st["stage"])
        path = os.path.join(parts_dir, st["name"], "model.safetensors")
        write_stage_file(path, dims, int(st["start_layer"]), int(st["end_layer"]), stage == 0,
                         stage == n_stages - 1, get_layer, get_global)
        written.append(path)
    return written


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--config", required=True, help="inferd.yaml-format span config")
    ap.add_argument("--model", default=None, help="inferd_amd model key (default: from model_name)")
    ap.add_argument("--checkpoint", help="HF safetensors checkpoint directory")
    ap.add_argument("--synthetic-seed", type=int, help="use counter-generated weights")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    with open(a.config) as f:
        cfg = yaml.safe_load(f)
    from .partitioned_models import _model_key
    dims = MODELS[a.model or _model_key(cfg["model_name"])]
    if a.checkpoint:
        if not a.model:      # the checkpoint's own geometry (config.json) when it has one
            dims = checkpoint_dims(a.checkpoint, name=cfg["model_name"]) or dims
        gl, gg = hf_checkpoint_source(a.checkpoint)
    elif a.synthetic_seed is not None:
        gl, gg = synthetic_source(dims, a.synthetic_seed)
    else:
        raise SystemExit("need --checkpoint or --synthetic-seed")
    for p in split(cfg, dims, gl, gg, a.out):
        print("wrote", p)


def synthetic_source(dims: ModelDims, seed: int):
    """Counter-based weights materialised on the GPU by the engine's generator."""
    from . import _lib
    lib = _lib.load()
    from .runtime import SpanRuntime  # noqa: F401  (library must be loadable)
    scale_lin, scale_norm = 0.034641016151377546, 0.1

    def gen(tid, shape, norm):
        n = 1
        for s in shape:
            n *= s
        t = torch.empty(n, dtype=torch.bfloat16, device="cuda")
        _lib.check(lib.inferd_weightgen(t.data_ptr(), n, seed, tid, scale_norm if norm else scale_lin,
                                        1.0 if norm else 0.0, _lib.stream_ptr()))
        return t.reshape(shape).cpu()

    h, I, H, KV, d = dims.hidden, dims.intermediate, dims.heads, dims.kv_heads, dims.head_dim
    shapes = {"self_attn.q_proj.weight": (0, (H * d, h)), "self_attn.k_proj.weight": (1, (KV * d, h)),
              "self_attn.v_proj.weight": (2, (KV * d, h)), "self_attn.o_proj.weight": (3, (h, H * d)),
              "self_attn.q_norm.weight": (4, (d,)), "self_attn.k_norm.weight": (5, (d,)),
              "input_layernorm.weight": (6, (h,)), "post_attention_layernorm.weight": (7, (h,)),
              "mlp.gate_proj.weight": (8, (I, h)), "mlp.up_proj.weight": (9, (I, h)),
              "mlp.down_proj.weight": (10, (h, I))}

    def get_layer(i):
        return {k: gen(i * 16 + idx, shp, "norm" in k) for k, (idx, shp) in shapes.items()}

    def get_global(name):
        tid = {"embed_tokens": 0xFFFF0000, "norm": 0xFFFF0001, "lm_head": 0xFFFF0002}[name]
        shp = (h,) if name == "norm" else (dims.vocab, h)
        return gen(tid, shp, name == "norm")
    return get_layer, get_global


if __name__ == "__main__":
    main()
