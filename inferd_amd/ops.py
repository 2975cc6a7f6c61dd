"""torch.ops.inferd: the span engine's C-ABI registered as PyTorch-ROCm operators
(inferd_amd/csrc/torch_ops.cpp -> libinferd_torch.so, built in-tree with the engine) -- the
binding the node-facing host (runtime.py) drives the engine through.

    import inferd_amd.ops                      # registers torch.ops.inferd.* / torch.classes.inferd.*
    span = torch.ops.inferd.span_create(cfg, eps, theta, device)
    words, shape = torch.ops.inferd.kv_build_batch(table, seqs, n_new, device)
    torch.ops.inferd.span_forward(span, words, shape, ids, None, None, next_ids, logits)
    g = torch.classes.inferd.DecodeGraph(span, table, seqs, n_steps, ids, None, None, ids, None, device)
    g.launch()

Every op runs on torch's current HIP stream, checks its tensors against the batch shape and the
span's sizes, and raises RuntimeError with the library's message on a non-zero status.  There is
no fallback: a missing library raises at import."""
from __future__ import annotations

import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libinferd_torch.so")

if not os.path.exists(LIB_PATH):
    raise RuntimeError(f"libinferd_torch.so not built ({LIB_PATH}); run __graft_entry__.build()")
from . import _lib  # noqa: E402  (checks the engine library's ABI version first)

_lib.load()
torch.ops.load_library(LIB_PATH)
ops = torch.ops.inferd

OPS = ("span_create", "span_destroy", "span_config", "span_init_synthetic", "span_set_weight", "span_error_flags",
       "span_profile_start", "span_profile_stop", "span_forward", "span_lm_head", "span_head_shard", "argmax_combine",
       "dedicated_stream",
       "weightgen", "kv_create",
       "kv_destroy", "kv_reserve", "kv_advance", "kv_release", "kv_query", "kv_pages", "kv_free_pages",
       "kv_build_batch")
CLASSES = ("DecodeGraph",)
KV_PAGE = _lib.KV_PAGE              # tokens per KV page (INFERD_KV_PAGE_TOKENS)
PROF_CLASSES = _lib.PROF_CLASSES    # span_profile_stop's kernel classes (INFERD_PROF_* order)


def span_config(dims, first_layer: int, n_layers: int, *, has_embed: bool, has_lm_head: bool, kv_pages: int,
                max_tokens: int, max_seqs: int, max_positions: int, skip_first_attn: bool = False,
                skip_last_mlp: bool = False, gateup_split_first: int = 0, gateup_split_last: int = 0,
                o_split_first: bool = False, o_split_last: bool = False, qkv_split_first: bool = False,
                qkv_split_last: bool = False, head_first: int = 0, head_rows: int = 0,
                final_norm_out: bool = False) -> list:
    """The 25 config ints of span_create (InferdSpanConfig order)."""
    return [dims.hidden, dims.intermediate, dims.heads, dims.kv_heads, dims.head_dim, dims.vocab, first_layer,
            n_layers, int(has_embed), int(has_lm_head), max_positions, kv_pages, max_tokens, max_seqs,
            int(skip_first_attn), int(skip_last_mlp), int(gateup_split_first), int(gateup_split_last),
            int(o_split_first), int(o_split_last), int(qkv_split_first), int(qkv_split_last), int(head_first),
            int(head_rows), int(final_norm_out)]
