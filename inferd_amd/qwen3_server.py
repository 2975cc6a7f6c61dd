"""Drop-in for `models/qwen3/server/qwen3_server_module.py::Qwen3Server` on the gfx950 engine.

Same constructor `Qwen3Server(start_layer, end_layer)` and the same
`send(session_id, hidden_states, attention_mask, cache_position, position_embeddings)`
(qwen3_server_module.py:209-255).  The per-session `DynamicCache`
(`session_caches = defaultdict(DynamicCache)`, :220) becomes the span's paged KV pool:
prefill appends T tokens, each decode call appends one, positions continue from the
cached length (client.py:244-266).

Arguments the GPU path derives itself, checked (semantics.py) rather than ignored:
  * attention_mask -- must be the client's additive causal mask (client.py:221-224 for
    prefill, the all-zero (1,1,1,1) mask for decode, :249-250); causality over the cached
    prefix is implicit in the attention kernels.  Any other mask (padding, non-causal, a
    T > 1 call without one) raises ValueError: the reference would apply it;
  * position_embeddings -- must be (cos, sin) of the HF default rope at cache_position
    (client.py:56-71); the engine keeps the same table (bf16) on the device.  A shifted or
    non-default rotary raises ValueError.
`cache_position` must continue the session's cached length; anything else raises
(the reference would silently concatenate onto the cache).

Sessions are keyed exactly as the reference keys its caches, `None` included (ProcessLayer
maps an empty id to None, server.py:39, and every None call then shares that cache).
Unlike the reference, sessions can be released (`release(session_id)`), and `max_sessions`
evicts the least recently used one (a later call that continues an evicted session fails
its cache_position check).
"""
from __future__ import annotations

from collections import OrderedDict

import torch

from .runtime import MODELS, ModelDims, SpanRuntime
from .semantics import check_additive_causal_mask, check_rotary


class Qwen3Server:
    def __init__(self, start_layer: int, end_layer: int, *, model: str | ModelDims = "qwen3-0.6b",
                 weights: str = "synthetic:1234", kv_pages: int = 1024, max_tokens: int = 8192,
                 max_sessions: int | None = None, device="cuda"):
        dims = MODELS[model] if isinstance(model, str) else model
        self.dims = dims
        self.start_layer, self.end_layer = start_layer, end_layer
        self.device = torch.device(device)
        self.span = SpanRuntime(dims, start_layer, end_layer - start_layer + 1, has_embed=False,
                                has_lm_head=False, kv_pages=kv_pages, max_tokens=max_tokens, max_seqs=64,
                                device=self.device)
        self.max_sessions = max_sessions
        self._lru = OrderedDict()
        if weights.startswith("synthetic:"):
            self.span.init_synthetic(int(weights.split(":")[1]))
        else:
            self.load_layer_files(weights)

    def load_layer_files(self, pattern: str):
        """Per-layer state dicts `layer_XX.pt` (qwen3_server_module.py:227-235: the HF-hub
        files of Qwen3Config.HF_REPO_ID), loaded with weights_only=True (nothing in the file
        executes); `pattern` contains `{idx:02d}`, e.g. "/ckpt/layer_{idx:02d}.pt"."""
        for j, i in enumerate(range(self.start_layer, self.end_layer + 1)):
            sd = torch.load(pattern.format(idx=i), map_location="cpu", weights_only=True)
            self.span.load_layer_state_dict(j, sd)

    @property
    def session_caches(self):
        return self.span.sessions

    def _keys(self, session_id, B):
        # the reference keys DynamicCache by session_id -- None included: ProcessLayer maps an
        # empty id to None (server.py:39) and defaultdict caches under it (:220, :253)
        return [("srv", session_id, b) for b in range(B)]

    def release(self, session_id):
        for key in [k for k in self.span.sessions if isinstance(k, tuple) and len(k) == 3 and k[0] == "srv"
                    and k[1] == session_id]:
            self.span.release(key)
        self._lru.pop(session_id, None)

    def send(self, session_id, hidden_states, attention_mask=None, cache_position=None,
             position_embeddings=None, input_start_layer=None, input_end_layer=None):
        """qwen3_server_module.py:237-255: hidden (B,T,h) -> hidden (B,T,h) through the span,
        appending T tokens to each of the B rows' caches of `session_id`."""
        B, T, h = hidden_states.shape
        keys = self._keys(session_id, B)
        st = self.span.sessions.get(keys[0])
        past = 0 if st is None else st.length
        if cache_position is not None:
            cp = torch.as_tensor(cache_position).reshape(-1).tolist()
            if cp != list(range(past, past + T)):
                raise ValueError(f"cache_position {cp[:3]}... does not continue session {session_id!r} "
                                 f"(cached length {past})")
        check_additive_causal_mask(attention_mask, B, T, past)
        check_rotary(position_embeddings, torch.arange(past, past + T), self.dims.rope_theta, self.dims.head_dim)
        if self.max_sessions is not None and session_id not in self._lru and len(self._lru) >= self.max_sessions:
            old, _ = self._lru.popitem(last=False)
            self.release(old)
        self._lru[session_id] = True
        self._lru.move_to_end(session_id)
        out = self.span.forward([(k, T) for k in keys], x=hidden_states.reshape(B * T, h))
        self.span.check_errors()
        return out["hidden"].reshape(B, T, h)
