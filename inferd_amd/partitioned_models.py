"""Drop-in replacement of `petals/partitioned_models.py` backed by the gfx950 span engine.

Same module-level names and contracts as the reference, so node.py / task.py /
run_node.py can import from here unchanged:

  tensor_to_base64(tensor) -> {"b64", "dtype", "shape"}      partitioned_models.py:11-18
  base64_to_tensor(meta)   -> tensor                          :20-26
  build_decoder_attention_mask(attn_mask_2d)                   :28-35
  FirstStage / StageInner / LastStage  .forward(model_in, decoder_attn_mask, position_ids)
                                                               :40-97
  PartitionedQwen2(model_name, num_stages, stage, parts_path).forward(inputs: dict) -> dict
                                                               :102-168

Differences, all on purpose:
  * the stage modules own a SpanRuntime (HIP kernels through the C-ABI) instead of HF
    decoder layers; compute is bf16 on the GPU and there is no CPU fallback;
  * the codec also carries bf16 (dtype "bfloat16", raw 16-bit words) -- the reference's
    `.numpy()` raises on bf16;  fp32 payloads keep the reference format;
  * the decoder mask argument is accepted for API compatibility but not materialised:
    causality is implicit in the attention kernels (partitioned_models.py:139-143 only
    ever builds a full causal mask with positions 0..T-1);
  * parts_path is a stage file written by inferd_amd.split_model (safetensors, loaded
    with a loader that executes nothing) or "synthetic:<seed>" for the counter-based
    weights; the reference's pickled `torch.save(module)` (split_model.py:107) needs
    `weights_only=False` and is not loaded.
"""
from __future__ import annotations

import base64
import json
import os

import numpy as np
import torch

from .runtime import MODELS, ModelDims, SpanRuntime

_BF16 = "bfloat16"


# ------------------------------------------------------------------ wire codec
def tensor_to_base64(tensor: torch.Tensor) -> dict:
    """partitioned_models.py:11-18, plus bf16 as raw 16-bit words."""
    t = tensor.detach().cpu().contiguous()
    if t.dtype == torch.bfloat16:
        raw = t.view(torch.int16).numpy().tobytes()
        return {"b64": base64.b64encode(raw).decode("utf-8"), "dtype": _BF16, "shape": list(t.shape)}
    array = t.numpy()
    return {"b64": base64.b64encode(array.tobytes()).decode("utf-8"), "dtype": str(array.dtype),
            "shape": list(array.shape)}


def base64_to_tensor(meta: dict) -> torch.Tensor:
    """partitioned_models.py:20-26, plus dtype "bfloat16"."""
    data = base64.b64decode(meta["b64"])
    shape = tuple(meta["shape"])
    if meta["dtype"] == _BF16:
        arr = np.frombuffer(data, dtype=np.int16).reshape(shape).copy()
        return torch.from_numpy(arr).view(torch.bfloat16)
    arr = np.frombuffer(data, dtype=meta["dtype"]).reshape(shape).copy()
    return torch.from_numpy(arr)


def build_decoder_attention_mask(attn_mask_2d: torch.Tensor) -> torch.Tensor:
    """partitioned_models.py:28-35: (1,1,T,T) bool, True = attend (causal & padding)."""
    seq_len = attn_mask_2d.size(1)
    causal = torch.tril(torch.ones((seq_len, seq_len), device=attn_mask_2d.device, dtype=torch.bool))
    causal = causal.unsqueeze(0).unsqueeze(1)
    padding = attn_mask_2d.unsqueeze(1).unsqueeze(2).to(torch.bool)
    return padding & causal


# ------------------------------------------------------------------ stage modules
class _Stage:
    """Common part of the three stage modules: a SpanRuntime and the reference's
    forward(model_in, decoder_attn_mask, position_ids) contract (batch 1 rows per
    sequence, full recompute from the given positions)."""

    first = last = False

    def __init__(self, span: SpanRuntime):
        self.span = span

    def to(self, *a, **k):
        return self

    def eval(self):
        return self

    def __call__(self, *a, **k):
        return self.forward(*a, **k)

    def _run(self, model_in, position_ids):
        B, T = model_in.shape[0], model_in.shape[1]
        if position_ids is not None:
            pos = position_ids.reshape(-1, T)[0].tolist()
            if pos != list(range(T)):
                raise ValueError("stage modules recompute from position 0 (partitioned_models.py:139-143); "
                                 "use Qwen3Server.send for cached positions")
        reqs = [(None, T)] * B
        kw = dict(want_hidden=not self.last, want_logits=self.last, want_next_ids=self.last)
        if self.first:
            out = self.span.forward(reqs, ids=model_in.reshape(-1), **kw)
        else:
            out = self.span.forward(reqs, x=model_in.reshape(B * T, -1), **kw)
        if self.last:
            # greedy ids from the engine's own argmax (bf16 logits, lowest index on ties,
            # = torch.argmax at partitioned_models.py:162)
            self.last_next_ids = out["next_ids"]
            return out["logits"].reshape(B, 1, -1)   # last position only (see LastStage)
        return out["hidden"].reshape(B, T, -1)


class FirstStage(_Stage):
    """partitioned_models.py:40-57: ids (B,T) -> hidden (B,T,h)."""
    first = True


class StageInner(_Stage):
    """partitioned_models.py:60-75: hidden (B,T,h) -> hidden (B,T,h)."""


class LastStage(_Stage):
    """partitioned_models.py:78-97: hidden (B,T,h) -> logits.  The reference computes
    lm_head over all T rows and then uses only the last (:96, :162); this returns the
    last row's logits as (B,1,V), which is everything `forward` consumes."""
    last = True


class FirstLastStage(_Stage):
    """A single span holding the whole model (ids -> last-row logits)."""
    first = last = True

    def forward(self, model_in, decoder_attn_mask=None, position_ids=None):
        return self._run(model_in, position_ids)


for _cls in (FirstStage, StageInner, LastStage):
    _cls.forward = lambda self, model_in, decoder_attn_mask=None, position_ids=None: self._run(model_in, position_ids)


# ------------------------------------------------------------------ stage files
def load_stage(parts_path: str, model_name: str, num_stages: int, stage: int, device) -> _Stage:
    """Build the stage module of `parts_path`:
      * "synthetic:<seed>[:<model>:<start>:<end>]" -- counter-based weights (no checkpoint)
      * a .safetensors stage file written by inferd_amd.split_model (metadata: model dims,
        start/end layer, roles)."""
    if parts_path.startswith("synthetic:"):
        bits = parts_path.split(":")
        seed = int(bits[1])
        dims = MODELS[bits[2] if len(bits) > 2 else _model_key(model_name)]
        if len(bits) > 4:
            start, end = int(bits[3]), int(bits[4])
        else:
            per = dims.layers // num_stages
            start = stage * per
            end = dims.layers - 1 if stage == num_stages - 1 else start + per - 1
        first, last = stage == 0, stage == num_stages - 1
        span = SpanRuntime(dims, start, end - start + 1, has_embed=first, has_lm_head=last, device=device)
        span.init_synthetic(seed)
        return _make_stage(span, first, last)
    from safetensors import safe_open
    with safe_open(parts_path, framework="pt", device="cpu") as f:
        meta = f.metadata()
        dims = ModelDims(**json.loads(meta["dims"]))
        start, end = int(meta["start_layer"]), int(meta["end_layer"])
        first, last = meta["first"] == "1", meta["last"] == "1"
        span = SpanRuntime(dims, start, end - start + 1, has_embed=first, has_lm_head=last, device=device)
        # norm weights first: the span folds them into the projections packed after them
        for key in sorted(f.keys(), key=lambda k: 0 if k.endswith("norm.weight") else 1):
            t = f.get_tensor(key)
            if key.startswith("layers."):
                _, j, *rest = key.split(".")
                span.set_weight(int(j), rest[-2], t)
            else:
                span.set_weight(-1, {"embed.weight": "embed_tokens", "norm.weight": "norm",
                                     "lm_head.weight": "lm_head"}[key], t)
    return _make_stage(span, first, last)


def _make_stage(span, first, last):
    if first and last:
        return FirstLastStage(span)
    return FirstStage(span) if first else (LastStage(span) if last else StageInner(span))


def _model_key(model_name: str) -> str:
    n = model_name.lower()
    for k in ("32b", "8b", "0.6b"):
        if k in n:
            return f"qwen3-{k}"
    return "qwen3-0.6b"


class _OfflineTokenizer:
    """Stand-in when no local tokenizer files exist: ids in, `<id>` strings out."""

    def decode(self, token_id):
        return f"<{token_id}>"

    def __call__(self, text, return_tensors=None):
        raise RuntimeError("no tokenizer available offline: send {'generated_ids': [...]} instead of text")


def _load_tokenizer(model_name):
    try:
        from transformers import AutoTokenizer
        return AutoTokenizer.from_pretrained(model_name, local_files_only=True)
    except Exception:
        return _OfflineTokenizer()


# ------------------------------------------------------------------ node-facing API
class PartitionedQwen2:
    """partitioned_models.py:102-168 -- same constructor, same forward(dict) -> dict."""

    def __init__(self, model_name: str, num_stages: int, stage: int, parts_path: str):
        self.stage = stage
        self.num_stages = num_stages
        self.parts_path = parts_path
        if not torch.cuda.is_available():
            raise RuntimeError("PartitionedQwen2 (inferd_amd) runs on an MI355X GPU; no CPU path")
        self.device = torch.device("cuda")
        if stage == 0 or stage == num_stages - 1:
            self.tokenizer = _load_tokenizer(model_name)
        self.model = load_stage(parts_path, model_name, num_stages, stage, self.device)

    def _prepare_inputs(self, input_data):
        """partitioned_models.py:119-137."""
        if self.stage == 0:
            if isinstance(input_data, str):
                ids = self.tokenizer(input_data, return_tensors="pt").input_ids
                return ids.reshape(-1).tolist(), ids
            if "prompt" in input_data:
                ids = self.tokenizer(input_data["prompt"], return_tensors="pt").input_ids
                return ids.reshape(-1).tolist(), ids
            if "generated_ids" in input_data:
                lst = input_data["generated_ids"]
                return lst, torch.tensor([lst], dtype=torch.long)
        if "hidden_meta" in input_data:
            hidden = base64_to_tensor(input_data["hidden_meta"])
            return input_data.get("generated_ids"), hidden
        raise RuntimeError(f"Bad input for stage {self.stage}: {input_data!r}")

    def forward(self, inputs: dict) -> dict:
        """partitioned_models.py:145-168 (same output schema)."""
        gen_ids, model_in = self._prepare_inputs(inputs)
        T = model_in.size(1)
        pos = torch.arange(T).unsqueeze(0)
        with torch.no_grad():
            out = self.model(model_in, None, pos)
        if self.stage < self.num_stages - 1:
            if self.stage == 0:
                return {"hidden_meta": tensor_to_base64(out), "generated_ids": gen_ids}
            return {"hidden_meta": tensor_to_base64(out)}
        token_id = int(self.model.last_next_ids[0].item())
        return {"next_token_id": token_id, "next_token_str": self.tokenizer.decode(token_id),
                "generated_ids": list(gen_ids) + [token_id]}
