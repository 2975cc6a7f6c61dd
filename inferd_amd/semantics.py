"""Checks that a caller's attention mask and rotary tables are the ones the engine computes.

The span engine attends causally over each sequence's cached prefix and rotates q/k with its
own table of the HF default rope (cos/sin[max_pos][64] bf16, span.hip).  The reference applies
whatever the caller hands it:
  * the petals stage modules take a bool mask, True = attend, consumed by HF SDPA
    (petals/partitioned_models.py:28-35, :47-97) -- `build_decoder_attention_mask` also folds a
    2-D padding mask into it;
  * Qwen3Server.send adds an additive mask to the scores, sliced to the key count
    (eager_attention_forward, qwen3_server_module.py:80-82), and rotates with the (cos, sin) it
    is given (:141-142, :150-158).
On the reference's own callers these are always the causal / zero masks of
partitioned_models.py:139-143 and client.py:221-224, :249-250 and the default rope at
cache_position (client.py:56-71, :226), which the engine reproduces.  Anything else would get a
silently different answer, so it is rejected here with ValueError before any kernel runs.
"""
from __future__ import annotations

import torch

# an additive mask entry at a masked-out key must drive its softmax weight to exactly 0: the
# client's finfo(dtype).min, -inf, or anything at or below float16's lowest finite value
MASKED_MAX = -65504.0


def allowed_keys(T: int, past: int, device=None) -> torch.Tensor:
    """(T, past + T) bool: query i (position past + i) may attend keys 0 .. past + i."""
    q = torch.arange(T, device=device)[:, None] + past
    return torch.arange(past + T, device=device)[None, :] <= q


def _as_4d(mask: torch.Tensor, B: int, T: int, K: int, what: str) -> torch.Tensor:
    if mask.dim() != 4:
        raise ValueError(f"{what}: a 4-D mask (batch, 1 | heads, queries, keys) is expected, got {tuple(mask.shape)}")
    m = mask[..., :K]
    try:
        return torch.broadcast_to(m, (B if m.shape[0] != 1 else 1, m.shape[1], T, K))
    except RuntimeError as e:
        raise ValueError(f"{what}: mask {tuple(mask.shape)} does not broadcast to {T} queries x {K} keys") from e


def check_bool_causal_mask(mask, B: int, T: int, what: str = "decoder_attn_mask") -> None:
    """A petals stage-module mask (True = attend, HF SDPA): it must be the full causal mask of
    positions 0..T-1 -- `build_decoder_attention_mask` of an all-ones 2-D mask
    (partitioned_models.py:139-143).  A padding mask or any non-causal pattern raises.  A float
    mask is taken as additive (what SDPA does with one) and checked like Qwen3Server's."""
    if mask is None:
        return
    mask = torch.as_tensor(mask)
    if mask.dtype != torch.bool:
        return check_additive_causal_mask(mask, B, T, 0, what)
    m = _as_4d(mask, B, T, T, what)
    if not bool((m == allowed_keys(T, 0, m.device)).all()):
        raise ValueError(f"{what}: only the full causal mask (no padding) is supported -- the engine attends every "
                         f"earlier position of the sequence (partitioned_models.py:28-35 with an all-ones padding mask)")


def check_additive_causal_mask(mask, B: int, T: int, past: int, what: str = "attention_mask") -> None:
    """Qwen3Server.send's additive mask (sliced to past + T keys like eager_attention_forward,
    qwen3_server_module.py:80-82): 0 at every key a query may attend (its cached prefix and the
    call's earlier positions) and <= MASKED_MAX at every later key.  None is accepted for a
    one-token call only: with no mask the reference lets a T > 1 call attend its own future
    positions."""
    if mask is None:
        if T > 1:
            raise ValueError(f"{what}=None: the reference adds no mask, so a {T}-token call would attend its own "
                             f"later positions; the engine is causal -- pass the client's causal mask "
                             f"(client.py:221-224)")
        return
    mask = torch.as_tensor(mask)
    if not mask.is_floating_point():
        raise ValueError(f"{what}: an additive floating-point mask is expected (qwen3_server_module.py:80-82 adds "
                         f"it to the scores), got {mask.dtype}")
    K = past + T
    m = _as_4d(mask, B, T, K, what).float()
    ok = torch.where(allowed_keys(T, past, m.device), m == 0, m <= MASKED_MAX)
    if not bool(ok.all()):
        raise ValueError(f"{what}: only the causal mask over the cached prefix is supported (0 at keys <= the "
                         f"query's position, finfo.min after it: client.py:221-224, :249-250)")


def default_rope(theta: float, positions: torch.Tensor, dtype=torch.bfloat16, head_dim: int = 128):
    """HF default rotary embedding at `positions` (client.py:39-71: fp32 inv_freq and freqs,
    cat(freqs, freqs), cos / sin, cast to the activation dtype): (cos, sin) [..., head_dim]."""
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.int64).float() / head_dim))
    freqs = positions.float()[..., None] * inv
    emb = torch.cat((freqs, freqs), dim=-1)
    return emb.cos().to(dtype), emb.sin().to(dtype)


def check_rotary(position_embeddings, positions, theta: float, head_dim: int = 128,
                 what: str = "position_embeddings") -> None:
    """(cos, sin) as Qwen3Server.send receives them ((B | 1, T, head_dim), client.py:226) must be
    the default rope at `positions` (the engine rotates with its own table of it): within two
    bf16 ulps of unit magnitude (1/128), which any shifted, scaled or non-default rotary misses
    on its high-frequency dimensions."""
    if position_embeddings is None:
        return
    cos, sin = position_embeddings
    cos, sin = torch.as_tensor(cos), torch.as_tensor(sin)
    pos = torch.as_tensor(positions).reshape(-1).cpu()
    T = pos.numel()
    rc, rs = default_rope(theta, pos, torch.float32, head_dim)
    for name, got, ref in (("cos", cos, rc), ("sin", sin, rs)):
        if got.shape[-1] != head_dim or got.shape[-2] != T:
            raise ValueError(f"{what}: {name} of shape {tuple(got.shape)}, expected (.., {T}, {head_dim})")
        err = (got.detach().float().cpu().reshape(-1, T, head_dim) - ref).abs().max().item()
        if err > 1.0 / 128:
            raise ValueError(f"{what}: {name} differs from the default rope at cache_position by {err:.3g} -- the "
                             f"engine rotates with its own table of the HF default rope (client.py:56-71)")
