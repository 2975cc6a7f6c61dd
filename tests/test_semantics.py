"""inferd_amd/semantics.py on CPU: which masks and rotary tables the engine accepts.

The engine attends causally over the cached prefix with its own default-rope table; the
reference applies whatever mask and (cos, sin) it is given (qwen3_server_module.py:80-82,
:141-142; petals/partitioned_models.py:28-35).  Accepted = exactly the inputs the reference's own
callers build (client.py:221-226, :249-250; partitioned_models.py:139-143)."""
import pytest
import torch

from inferd_amd import semantics as S
from oracle import qwen3_ref as R

D = R.CONFIGS["qwen3-0.6b"]
MIN = torch.finfo(torch.bfloat16).min


def client_prefill_mask(B, T, dtype=torch.bfloat16):
    """client.py:221-224"""
    tril = torch.tril(torch.ones(T, T, dtype=dtype))
    return ((1.0 - tril) * torch.finfo(dtype).min)[None, None].expand(B, 1, T, T)


def test_bool_causal_mask():
    from inferd_amd.partitioned_models import build_decoder_attention_mask
    T = 7
    S.check_bool_causal_mask(build_decoder_attention_mask(torch.ones(1, T, dtype=torch.long)), 1, T)
    S.check_bool_causal_mask(None, 1, T)
    pad = torch.ones(1, T, dtype=torch.long)
    pad[0, :2] = 0
    with pytest.raises(ValueError):
        S.check_bool_causal_mask(build_decoder_attention_mask(pad), 1, T)
    with pytest.raises(ValueError):
        S.check_bool_causal_mask(torch.ones(1, 1, T, T, dtype=torch.bool), 1, T)   # non-causal
    S.check_bool_causal_mask(client_prefill_mask(1, T, torch.float32), 1, T)       # additive form


def test_additive_masks_of_the_client():
    for dt in (torch.bfloat16, torch.float32):
        S.check_additive_causal_mask(client_prefill_mask(2, 9, dt), 2, 9, 0)
    S.check_additive_causal_mask(torch.zeros(1, 1, 1, 1), 1, 1, 40)                # decode token
    S.check_additive_causal_mask(None, 1, 1, 40)
    with pytest.raises(ValueError):
        S.check_additive_causal_mask(None, 1, 5, 0)
    # a prefill that continues a cached prefix: the mask must span past + T keys
    past, T = 4, 3
    m = torch.zeros(1, 1, T, past + T)
    m[0, 0][~S.allowed_keys(T, past)] = float("-inf")
    S.check_additive_causal_mask(m, 1, T, past)
    with pytest.raises(ValueError):      # the client's T x T mask cannot address the cached keys
        S.check_additive_causal_mask(client_prefill_mask(1, T), 1, T, past)
    bad = client_prefill_mask(1, 6).clone()
    bad[..., 0] = MIN                    # padding on key 0
    with pytest.raises(ValueError):
        S.check_additive_causal_mask(bad, 1, 6, 0)
    with pytest.raises(ValueError):
        S.check_additive_causal_mask(torch.zeros(1, 1, 6, 6), 1, 6, 0)              # non-causal
    with pytest.raises(ValueError):
        S.check_additive_causal_mask(torch.ones(1, 1, 6, 6, dtype=torch.bool), 1, 6, 0)
    with pytest.raises(ValueError):     # 3-row batch mask for 2 rows
        S.check_additive_causal_mask(client_prefill_mask(3, 6), 2, 6, 0)


def test_rotary_default_matches_oracle_and_rejects_others():
    pos = torch.arange(100, 140)
    for dt in (torch.bfloat16, torch.float32):
        cos, sin = R.rope_cos_sin(D, pos[None], dt)                # HF / client.py:56-71
        rc, rs = S.default_rope(D.rope_theta, pos, dt)
        assert torch.equal(rc, cos[0]) and torch.equal(rs, sin[0])
        S.check_rotary((cos, sin), pos, D.rope_theta)
    cos, sin = R.rope_cos_sin(D, (pos + 1)[None], torch.bfloat16)
    with pytest.raises(ValueError):
        S.check_rotary((cos, sin), pos, D.rope_theta)
    cos, sin = R.rope_cos_sin(D, pos[None], torch.bfloat16)
    with pytest.raises(ValueError):
        S.check_rotary((cos, sin * 1.1), pos, D.rope_theta)
    with pytest.raises(ValueError):     # another base (rope_theta 1e4)
        S.check_rotary(S.default_rope(1e4, pos), pos, D.rope_theta)
    S.check_rotary(None, pos, D.rope_theta)
