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
    `.numpy()` raises on bf16;  fp32 payloads keep the reference format, and
    INFERD_WIRE_DTYPE=float32 makes a GPU stage emit fp32 for a stock reference node
    downstream (partitioned_models.py:20-26 cannot decode bf16);
  * the decoder mask is not materialised: causality is implicit in the attention kernels
    (partitioned_models.py:139-143 only ever builds the full causal mask of positions
    0..T-1); any other mask -- padding, non-causal -- raises ValueError (semantics.py) instead
    of being silently ignored;
  * parts_path is a stage file written by inferd_amd.split_model (safetensors, loaded
    with a loader that executes nothing) or "synthetic:<seed>" for the counter-based
    weights; the reference's pickled `torch.save(module)` (split_model.py:107) is converted
    once by `python -m inferd_amd.convert_parts` (an inert unpickler: nothing in the file
    runs) instead of being loaded;
  * an optional "session_id" in the input dict keeps K/V per sequence on every stage
    (PartitionedQwen2 docstring); without it the protocol is the reference's, unchanged.
"""
from __future__ import annotations

import base64
import json
import os
from collections import OrderedDict

import numpy as np
import torch

from .runtime import MODELS, ModelDims, SpanRuntime
from .semantics import check_bool_causal_mask

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
    forward(model_in, decoder_attn_mask, position_ids) contract (full recompute from
    position 0 of B sequences of T rows)."""

    first = last = False

    def __init__(self, span: SpanRuntime):
        self.span = span
        self.last_next_ids = self.last_logits = None

    def to(self, *a, **k):
        return self

    def eval(self):
        return self

    def __call__(self, *a, **k):
        return self.forward(*a, **k)

    def forward(self, model_in, decoder_attn_mask=None, position_ids=None):
        B, T = model_in.shape[0], model_in.shape[1]
        check_bool_causal_mask(decoder_attn_mask, B, T)
        if position_ids is not None:
            pos = position_ids.reshape(-1, T)[0].tolist()
            if pos != list(range(T)):
                raise ValueError("stage modules recompute from position 0 (partitioned_models.py:139-143); "
                                 "use Qwen3Server.send or a session_id for cached positions")
        out = self.run([(None, T)] * B, model_in, all_logits=True)
        return out.reshape(B, T, -1)

    def run(self, requests, model_in, all_logits=False, want_hidden=None):
        """requests: [(session key or None, new rows)] over the rows of model_in (ids (1,M) /
        (M,) on the first span, hidden (.., M, h) otherwise).  Returns the hidden rows (M, h),
        or on the last span the logits: (M, V) with all_logits, else the last row of each
        request (n, V); greedy ids of those last rows land in self.last_next_ids."""
        kw = {}
        if self.first:
            kw["ids"] = model_in.reshape(-1)
        else:
            kw["x"] = model_in.reshape(-1, self.span.dims.hidden)
        if not self.last:
            return self.span.forward(requests, want_hidden=True, **kw)["hidden"]
        out = self.span.forward(requests, want_hidden=all_logits, want_logits=not all_logits, want_next_ids=True,
                                **kw)
        # greedy ids from the engine's own argmax (bf16 logits, lowest index on ties,
        # = torch.argmax at partitioned_models.py:162)
        self.last_next_ids = out["next_ids"]
        if not all_logits:
            self.last_logits = out["logits"]
            return out["logits"]
        return self.span.lm_head(out["hidden"])


class FirstStage(_Stage):
    """partitioned_models.py:40-57: ids (B,T) -> hidden (B,T,h)."""
    first = True


class StageInner(_Stage):
    """partitioned_models.py:60-75: hidden (B,T,h) -> hidden (B,T,h)."""


class LastStage(_Stage):
    """partitioned_models.py:78-97: hidden (B,T,h) -> logits (B,T,V) (final norm + lm_head on
    every row, as the reference).  PartitionedQwen2.forward needs only the last row and calls
    `run`, which computes that row alone."""
    last = True


class FirstLastStage(_Stage):
    """A single span holding the whole model (ids -> logits)."""
    first = last = True


# ------------------------------------------------------------------ stage files
def _span_kwargs():
    """Workspace of a node's span: max_tokens rows per engine call (longer prompts run in
    chunks through their own pages), a KV pool for a full-length prompt
    (MAX_POSITION_EMBEDDINGS = 40960, qwen3_config.py:14) plus sessions."""
    return dict(kv_pages=int(os.environ.get("INFERD_KV_PAGES", 1024)),
                max_tokens=int(os.environ.get("INFERD_MAX_TOKENS", 4096)), max_seqs=64)


def load_stage(parts_path: str, model_name: str, num_stages: int, stage: int, device) -> _Stage:
    """Build the stage module of `parts_path`:
      * "synthetic:<seed>[:<model>:<start>:<end>[:<profile>]]" -- counter-based weights (no
        checkpoint); profile "peaked" = the large-margin embed / lm_head of oracle/weightgen.py
      * a .safetensors stage file written by inferd_amd.split_model (metadata: model dims,
        start/end layer, roles)."""
    if parts_path.startswith("synthetic:"):
        bits = parts_path.split(":")
        seed = int(bits[1])
        dims = MODELS[bits[2] if len(bits) > 2 and bits[2] else _model_key(model_name)]
        if len(bits) > 4:
            start, end = int(bits[3]), int(bits[4])
        else:
            per = dims.layers // num_stages
            start = stage * per
            end = dims.layers - 1 if stage == num_stages - 1 else start + per - 1
        profile = bits[5] if len(bits) > 5 else "random"
        first, last = stage == 0, stage == num_stages - 1
        span = SpanRuntime(dims, start, end - start + 1, has_embed=first, has_lm_head=last, device=device,
                           **_span_kwargs())
        span.init_synthetic(seed, profile)
        return _make_stage(span, first, last)
    from safetensors import safe_open
    with safe_open(parts_path, framework="pt", device="cpu") as f:
        meta = f.metadata()
        dims = ModelDims(**json.loads(meta["dims"]))
        start, end = int(meta["start_layer"]), int(meta["end_layer"])
        first, last = meta["first"] == "1", meta["last"] == "1"
        span = SpanRuntime(dims, start, end - start + 1, has_embed=first, has_lm_head=last, device=device,
                           **_span_kwargs())
        for key in f.keys():
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
    """runtime.MODELS key of a model name for synthetic stages (no checkpoint): the Qwen3 size in
    the name, else qwen3-0.6b -- the reference's default config names Qwen/Qwen2-0.5B
    (petals/inferd.yaml:1); the engine runs the Qwen3 layer of the same scale.  Checkpoints carry
    their own geometry (split_model.checkpoint_dims), which refuses non-Qwen3 architectures."""
    n = model_name.lower()
    for k in ("32b", "8b", "0.6b"):
        if k in n:
            return f"qwen3-{k}"
    if n in MODELS:
        return n
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
    """partitioned_models.py:102-168 -- same constructor, same forward(dict) -> dict.

    Stateless (the reference's protocol, unchanged): every call recomputes the whole
    sequence from position 0 (send_message.py:46-60 resends all generated ids).

    Session-cached (optional): an input dict that carries "session_id" keeps
    that sequence's K/V on every stage, so a step costs O(new tokens) instead of O(T):
      * stage 0 still receives the full `generated_ids` (the client loop is unchanged); it
        runs only the ids past the ones it has cached for the session (a list that does not
        extend the cached prefix restarts the session);
      * hidden_meta then carries only the new rows, plus "session_id" and "past_len" (the
        position of its first row) for the next stage, which appends them to its own pages;
      * {"session_id": s, "close_session": True} releases the session along the chain.
    Sessions beyond `max_sessions` (INFERD_MAX_SESSIONS, default 64) or a full KV pool evict
    the least recently used one (the reference's session caches are never freed,
    qwen3_server_module.py:220).
    A downstream stage that no longer holds a session's rows (evicted under another pool size
    or session cap, restarted) answers {"session_id", "session_lost": True, "generated_ids"}
    instead of raising; later stages pass that answer through (dropping their own copy), so it
    reaches the client as the chain's result.  The client resends the same generated_ids with
    "restart_session": True, and stage 0 recomputes the session from position 0 (every
    downstream stage then restarts it too: past_len 0)."""

    def __init__(self, model_name: str, num_stages: int, stage: int, parts_path: str):
        self.stage = stage
        self.num_stages = num_stages
        self.parts_path = parts_path
        if not torch.cuda.is_available():
            raise RuntimeError("PartitionedQwen2 (inferd_amd) runs on an MI355X GPU; no CPU path")
        self.device = torch.device("cuda", torch.cuda.current_device())
        if stage == 0 or stage == num_stages - 1:
            self.tokenizer = _load_tokenizer(model_name)
        self.model = load_stage(parts_path, model_name, num_stages, stage, self.device)
        self.span = self.model.span
        self.wire_dtype = os.environ.get("INFERD_WIRE_DTYPE", _BF16)
        self.max_sessions = int(os.environ.get("INFERD_MAX_SESSIONS", 64))
        self._sessions = OrderedDict()   # session_id -> ids cached (stage 0) / rows cached

    @property
    def _last(self):
        return self.stage == self.num_stages - 1

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
                if isinstance(lst, int):          # a 1-token prompt arrives as an int (:124,:128)
                    lst = [lst]
                return lst, torch.tensor([lst], dtype=torch.long)
        if "hidden_meta" in input_data:
            hidden = base64_to_tensor(input_data["hidden_meta"])
            return input_data.get("generated_ids"), hidden
        raise RuntimeError(f"Bad input for stage {self.stage}: {input_data!r}")

    def _encode(self, hidden):
        return tensor_to_base64(hidden.float() if self.wire_dtype == "float32" else hidden)

    def _output(self, out, gen_ids, rows, extra):
        if not self._last:
            res = {"hidden_meta": self._encode(out.reshape(1, rows, -1))}
            if self.stage == 0:
                res["generated_ids"] = gen_ids
            res.update(extra)
            return res
        token_id = int(self.last_next_ids[0].item())
        res = {"next_token_id": token_id, "next_token_str": self.tokenizer.decode(token_id),
               "generated_ids": list(gen_ids if gen_ids is not None else []) + [token_id]}
        res.update(extra)
        return res

    def forward(self, inputs: dict) -> dict:
        """partitioned_models.py:145-168 (same output schema)."""
        if isinstance(inputs, dict) and "session_id" in inputs:
            return self._forward_session(inputs)
        gen_ids, model_in = self._prepare_inputs(inputs)
        T = model_in.size(1)
        out = self._run([(None, T)], model_in)
        return self._output(out, gen_ids, T, {})

    # compute / cache hooks (inferd_amd.node_group runs them across a multi-GPU group)
    @torch.no_grad()
    def _run(self, requests, model_in):
        out = self.model.run(requests, model_in)
        self.span.check_errors()
        return out

    def _release(self, key):
        self.span.release(key)

    def _cached_len(self, key):
        st = self.span.sessions.get(key)
        return 0 if st is None else st.length

    @property
    def last_next_ids(self):
        return self.model.last_next_ids

    # ---------------------------------------------------------------- sessions
    def _touch(self, sid, value):
        self._sessions[sid] = value
        self._sessions.move_to_end(sid)
        while len(self._sessions) > self.max_sessions:
            old, _ = self._sessions.popitem(last=False)
            self._release(("sess", old))

    def close_session(self, sid):
        self._sessions.pop(sid, None)
        self._release(("sess", sid))

    def _forward_session(self, inputs):
        sid = inputs["session_id"]
        if inputs.get("close_session"):
            self.close_session(sid)
            return {"session_id": sid, "close_session": True} if not self._last else \
                {"session_id": sid, "closed": True}
        if inputs.get("session_lost"):         # an upstream stage lost it: pass the answer on
            self.close_session(sid)
            return {"session_id": sid, "session_lost": True, "generated_ids": inputs.get("generated_ids")}
        gen_ids, model_in = self._prepare_inputs(inputs)
        key = ("sess", sid)
        past = self._cached_len(key)
        if self.stage == 0:
            seen = self._sessions.get(sid)
            ids = model_in.reshape(-1).tolist()
            if inputs.get("restart_session") or seen is None or past != len(seen) or ids[:past] != seen or \
                    len(ids) <= past:
                self.close_session(sid)        # not a continuation (or the client asks): restart from 0
                past = 0
            new = model_in[:, past:]
        else:
            first_pos = int(inputs.get("past_len", 0))
            if first_pos != past:
                self.close_session(sid)
                if first_pos != 0:             # rows past a prefix this stage no longer holds
                    return {"session_id": sid, "session_lost": True, "generated_ids": gen_ids}
                past = 0
            new = model_in
        n = new.shape[1]
        while True:   # make room first: a full pool evicts the least recently used session
            try:
                self.span.reserve(key, n)
                break
            except RuntimeError as e:
                if "KV pool exhausted" not in str(e) or not self._evict_other(sid):
                    raise
        out = self._run([(key, n)], new)
        self._touch(sid, (model_in.reshape(-1).tolist() if self.stage == 0 else past + n))
        return self._output(out, gen_ids, n, {"session_id": sid, "past_len": past})

    def _evict_other(self, sid):
        for old in list(self._sessions):
            if old != sid:
                self.close_session(old)
                return True
        return False
