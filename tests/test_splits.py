"""Stage splits of the span pipeline (inferd_amd/pipeline.py) on CPU: layer, half-layer and
gate/up boundaries cover the model exactly once, respect the span engine's constraints
(include/inferd_span.h InferdSpanConfig), and the hand-off record sizes match the engine's."""
import pytest

from inferd_amd import pipeline as P
from inferd_amd.runtime import MODELS

D8 = MODELS["qwen3-8b"]


def _cover(ranges, n_layers, intermediate):
    """every half-layer unit once, in order; a gate/up column boundary continues exactly where
    the previous stage stopped"""
    u = 0
    prev_col = 0
    for i, r in enumerate(ranges):
        assert r.first_unit == u, (i, r)
        assert r.first_col == prev_col, (i, r)
        assert r.first_col % 128 == 0 and r.last_col % 128 == 0
        assert 0 <= r.first_col < intermediate and 0 <= r.last_col < intermediate
        if r.first_col:
            assert r.skip_first_attn
        if r.last_col:
            assert r.skip_last_mlp
        u += r.n_units
        prev_col = r.last_col
    assert u == 2 * n_layers and prev_col == 0


@pytest.mark.parametrize("n", [1, 2, 4, 8])
def test_splits_cover_the_model(n):
    for ranges in (P.halves_split(D8.layers, n), P.gateup_split(D8.layers, n, D8.intermediate)):
        assert len(ranges) == n
        _cover(ranges, D8.layers, D8.intermediate)
    assert [r.label() for r in P.ranges_from_sizes([4.5, 4.5, 5, 5, 4.5, 5, 5, 2.5])][:2] == ["0..4a", "4m..8"]
    with pytest.raises(ValueError):
        P.ranges_from_sizes([4.25, 31.75])


def test_gateup_split_balances_better_than_halves():
    """On the cost model the gate/up boundaries lift the lowest stage's bytes-per-tick above the
    half-layer split's at 8 stages (what bench.py's stage_projection then measures)."""
    import bench

    def score(ranges):
        c = P.DECODE_US_8B
        t, b = [], []
        for i, r in enumerate(ranges):
            last = i == len(ranges) - 1
            n_attn = sum(1 for u in range(r.first_unit, r.first_unit + r.n_units) if u % 2 == 0)
            gu = P.DECODE_US_8B_GATEUP * (r.last_col - r.first_col) / D8.intermediate
            t.append(n_attn * c["attn_half"] + (r.n_units - n_attn) * c["mlp_half"] + gu + c["stage_norm"] +
                     (c["head"] if last else 0.0))
            b.append(bench.range_bytes(D8, r, 16, 2060, last))
        return min(b) / max(t)
    assert score(P.gateup_split(D8.layers, 8, D8.intermediate)) > score(P.halves_split(D8.layers, 8))


def test_record_sizes():
    assert P.record_elems(D8, 16) == 16 * 4096 + 16 * 12288
    assert P.record_elems(D8, 17) == 17 * 4096 + 32 * 12288
    assert P.handoff_elems(D8, 16, 0) == 16 * 4096
    assert P.handoff_elems(D8, 16, 2048) == 16 * 4096 + 16 * 2048      # one row tile: a prefix
    assert P.handoff_elems(D8, 20, 2048) == P.record_elems(D8, 20)     # several: the whole record
    r = P.StageRange(9, 10, 2048, 4096)
    assert r.span_kwargs() == {"skip_first_attn": True, "skip_last_mlp": True, "gateup_split_first": 2048,
                               "gateup_split_last": 4096}
    assert r.label() == "4m@2048..9a+4096"
    with pytest.raises(AssertionError):
        P.StageRange(8, 10, 2048, 0)          # a gate/up boundary refines a half boundary
