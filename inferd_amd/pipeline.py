"""Multi-GPU layer-span pipeline: one process per GPU, one span per process, hidden states
handed stage -> stage with RCCL send/recv over xGMI, greedy ids returned last -> first.

This replaces, inside one node, the reference's chain of HTTP hops between span nodes
(node.py:102-130 `send_to_next_node` POSTing base64 fp32 hidden states,
partitioned_models.py:11-26) with device-to-device p2p transfers of bf16 hidden
states.  Routing across nodes (DHT / path_finder / balancer) is untouched.

Schedule (lockstep ring).  Work items are (decode step k, microbatch m), linearised as
i = k * S + m for S stages and S microbatches in flight.  Stage s processes item i at
tick i + s.  At the start of every tick each stage runs ONE grouped exchange
(batch_isend_irecv): it sends the output it produced in the previous tick to its
successor and receives the input for this tick from its predecessor; the last stage's
successor is stage 0, which receives the greedy ids of item i - S (same microbatch, one
step earlier) exactly when it needs them.  Every transfer is produced one tick before it
is consumed, so in steady state all S stages compute every tick; grouping the send and
the recv of a tick into one exchange keeps two-rank rings (where both directions share
a communicator) deadlock-free.

Every microbatch owns fixed device buffers (ids / hidden in / hidden out / ids out), so
the decode compute of (stage, microbatch) is one replay of a captured HIP graph whose
first node advances that microbatch's positions on the device (runtime.DecodeGraph).
The compute of one item is delegated to an executor (SpanExecutor: the HIP span engine
on this rank's GPU); tests drive the same schedule on CPU ranks (gloo) with an oracle
executor.
"""
from __future__ import annotations

import sys
import time

import torch

from .runtime import KV_PAGE, DecodeGraph, ModelDims, SpanRuntime


def record_elems(dims, rows: int) -> int:
    """bf16 elements of a gate/up-boundary hand-off record of `rows` token rows: h1 [rows][hidden]
    then the SwiGLU product fragment-packed [rows rounded to 16][intermediate]
    (include/inferd_span.h InferdSpanConfig gateup_split_*)."""
    return rows * dims.hidden + (rows + 15) // 16 * 16 * dims.intermediate


def q_record_elems(dims, rows: int, pure: bool) -> int:
    """bf16 elements of a q/k/v|attention-boundary hand-off of `rows` token rows: x
    [rows][hidden], then -- a pure decode call -- the raw q/k/v rows [rows][(heads + 2 kv_heads)
    * head_dim] (InferdSpanConfig qkv_split_*)."""
    return rows * dims.hidden + (rows * (dims.heads + 2 * dims.kv_heads) * dims.head_dim if pure else 0)


def handoff_elems(dims, rows: int, col: int, o: bool = False, pure: bool = True, q: bool = False) -> int:
    """Elements of a hand-off that carry data (pure: a pure decode call, every sequence one new
    token): at an attention|o boundary (o) the whole record (o_record_elems, packed in a pure
    decode call of <= 64 rows); at a q/k/v|attention boundary (q) q_record_elems; else h1 alone
    (col = 0, a layer or half-layer boundary, or a call of more than 64 rows), else h1 plus the
    act columns [0, col) -- for <= 16 rows those are one contiguous prefix of the packed act (a
    16-row tile's columns [0, col) are its first 16 * col elements), for more rows the whole
    record."""
    if o:
        return o_record_elems(dims, rows, pure and rows <= 64)
    if q:
        return q_record_elems(dims, rows, pure)
    if not col or rows > 64:
        return rows * dims.hidden
    return rows * dims.hidden + 16 * col if rows <= 16 else record_elems(dims, rows)


def buffer_elems(dims, rows: int, col: int, o: bool = False, pure: bool = True, q: bool = False) -> int:
    """Elements of the buffer a stage boundary's hand-off lands in (the whole record, of which
    handoff_elems carries data; rows * hidden at a layer or half-layer boundary)."""
    if o:
        return o_record_elems(dims, rows, pure and rows <= 64)
    if q:
        return q_record_elems(dims, rows, pure)
    return record_elems(dims, rows) if col and rows <= 64 else rows * dims.hidden


def o_record_elems(dims, rows: int, packed: bool) -> int:
    """bf16 elements of an attention|o-boundary hand-off record of `rows` token rows: the layer's
    input residual x [rows][hidden], then the attention output [rows, or rows rounded to 16 when
    fragment-packed (a pure decode call)][heads * head_dim] (InferdSpanConfig o_split_*)."""
    return rows * dims.hidden + ((rows + 15) // 16 * 16 if packed else rows) * dims.heads * dims.head_dim


def pack_rows(t: torch.Tensor) -> torch.Tensor:
    """[rows, K] -> the fragment-packed layout of decode hand-offs (common.h packed_index: the
    16-row, 32-column tile (mt, kt) is 512 elements at (mt * K/32 + kt) * 512, element (r, c) of it
    at (c % 32 // 8) * 128 + r * 8 + c % 8), rows zero-padded to a multiple of 16.  Host side of
    the records' packed parts, for tests and CPU executors."""
    rows, K = t.shape
    R = (rows + 15) // 16 * 16
    p = torch.zeros(R, K, dtype=t.dtype, device=t.device)
    p[:rows] = t
    return p.view(R // 16, 16, K // 32, 4, 8).permute(0, 2, 3, 1, 4).reshape(-1)


def unpack_rows(flat: torch.Tensor, rows: int, K: int) -> torch.Tensor:
    """Inverse of pack_rows: the first `rows` rows [rows, K]."""
    R = (rows + 15) // 16 * 16
    return flat[:R * K].view(R // 16, K // 32, 4, 16, 8).permute(0, 3, 1, 2, 4).reshape(R, K)[:rows]


def even_split(n_layers: int, n: int):
    """[(first layer, layer count)] per stage, counts differing by at most one."""
    base, extra = divmod(n_layers, n)
    sizes = [base + (1 if i < extra else 0) for i in range(n)]
    return [(sum(sizes[:i]), k) for i, k in enumerate(sizes)]


def balanced_split(n_layers: int, n: int, layer_cost: float, head_cost: float = 0.0, embed_cost: float = 0.0):
    """[(first layer, layer count)] per stage minimising the slowest stage's cost, where a
    stage costs layer_cost per layer plus embed_cost on stage 0 and head_cost (final norm +
    lm_head + argmax) on the last stage; ties go to the split with the smallest sum of
    squared stage costs.  Every stage keeps at least one layer.

    A lockstep pipeline ticks at its slowest stage, so the even split that split_model.py's
    hand-written layer ranges would give (split_model.py:92-108, inferd.yaml) leaves every
    other stage idle for the lm_head's share of the last stage: at Qwen3-8B decode the
    lm_head reads V*h*2 = 1.24 GB, about 2.4 layers' worth of weights + KV."""
    assert 1 <= n <= n_layers
    INF = (float("inf"), float("inf"))
    # best[s][l]: (max cost, sum of squares) of stages 0..s-1 covering layers 0..l-1
    best = [[INF] * (n_layers + 1) for _ in range(n + 1)]
    cut = [[0] * (n_layers + 1) for _ in range(n + 1)]
    best[0][0] = (0.0, 0.0)
    for s in range(1, n + 1):
        for l in range(s, n_layers - (n - s) + 1):
            for j in range(s - 1, l):
                mx, sq = best[s - 1][j]
                if mx == float("inf"):
                    continue
                c = (l - j) * layer_cost + (embed_cost if s == 1 else 0.0) + (head_cost if s == n else 0.0)
                cand = (max(mx, c), sq + c * c)
                if cand < best[s][l]:
                    best[s][l], cut[s][l] = cand, j
    sizes, l = [], n_layers
    for s in range(n, 0, -1):
        j = cut[s][l]
        sizes.append(l - j)
        l = j
    sizes.reverse()
    return [(sum(sizes[:i]), k) for i, k in enumerate(sizes)]


class StageRange:
    """A stage's slice of the model in half-layer units: unit 2*l is layer l's attention half
    (input_layernorm .. o_proj + residual), unit 2*l + 1 its MLP half (post_attention_layernorm
    .. down_proj + residual), qwen3_server_module.py:179-206.  The reference cuts spans at
    layer boundaries only (split_model.py:92-108); a cut between the halves hands over the
    residual stream h1, a bf16 [tokens, hidden] tensor like a layer boundary's.
    first_col / last_col refine a half boundary into the layer's gate/up projection (decode
    calls; InferdSpanConfig gateup_split_*): the stage before it also computes gate/up columns
    [0, col), the stage after it the rest and the down projection, and the hand-off is h1 plus
    the packed SwiGLU product (a record).
    first_o / last_o: a boundary between layer l's attention and its o projection
    (InferdSpanConfig o_split_*): unit 2l then belongs to both stages -- the one before runs its
    norm, q/k/v and attention (its K/V live there), the one after its o projection -- and the
    hand-off is the record (x, attention output).  A first_o stage starts at unit 2l, a last_o
    stage ends after unit 2l.
    first_q / last_q: likewise a boundary between layer l's q/k/v projection and its attention
    (InferdSpanConfig qkv_split_*): the stage before runs the norm and q/k/v, the one after the
    attention (its K/V live there), o and the MLP; the hand-off is (x, the raw q/k/v rows) in a
    pure decode call, x alone otherwise."""
    __slots__ = ("first_unit", "n_units", "first_col", "last_col", "first_o", "last_o", "first_q", "last_q")

    def __init__(self, first_unit: int, n_units: int, first_col: int = 0, last_col: int = 0,
                 first_o: bool = False, last_o: bool = False, first_q: bool = False, last_q: bool = False):
        assert first_unit >= 0 and n_units >= 1
        self.first_unit, self.n_units = first_unit, n_units
        self.first_col, self.last_col = first_col, last_col
        self.first_o, self.last_o = bool(first_o), bool(last_o)
        self.first_q, self.last_q = bool(first_q), bool(last_q)
        assert not (first_o and first_q) and not (last_o and last_q)
        assert not first_col or self.skip_first_attn, "first_col refines a stage that starts at an MLP half"
        assert not last_col or self.skip_last_mlp, "last_col refines a stage that ends after an attention half"
        assert not (first_o or first_q) or first_unit % 2 == 0, "first_o / first_q: the stage starts in an attention unit"
        assert not (last_o or last_q) or (first_unit + n_units) % 2 == 1, \
            "last_o / last_q: the stage ends in an attention unit"
        assert not ((first_o or first_q) and (last_o or last_q) and n_units == 1), \
            "a stage that starts and ends inside one attention unit"

    @classmethod
    def layers(cls, first_layer: int, n_layers: int) -> "StageRange":
        return cls(2 * first_layer, 2 * n_layers)

    @classmethod
    def from_label(cls, label: str) -> "StageRange":
        """Inverse of label(): e.g. '4m@12032..9a+4096', '14o..18', '9m@768..14q'."""
        import re
        m = re.fullmatch(r"(\d+)(m?)(o?)(k?)(?:@(\d+))?\.\.(\d+)(a?)(q?)(v?)(?:\+(\d+))?", label)
        if not m:
            raise ValueError(f"not a stage label: {label}")
        l0, m0, o0, k0, c0, l1, a1, q1, v1, c1 = m.groups()
        first = 2 * int(l0) + (1 if m0 else 0)
        end = 2 * int(l1) + (1 if (a1 or q1 or v1) else 2)
        return cls(first, end - first, int(c0 or 0), int(c1 or 0), bool(o0), bool(q1), bool(k0), bool(v1))

    first_layer = property(lambda self: self.first_unit // 2)
    last_layer = property(lambda self: (self.first_unit + self.n_units - 1) // 2)
    n_layers = property(lambda self: self.last_layer - self.first_layer + 1)
    skip_first_attn = property(lambda self: self.first_unit % 2 == 1)
    skip_last_mlp = property(lambda self: (self.first_unit + self.n_units) % 2 == 1 and not (self.last_o or self.last_q))
    # the next stage's first_unit (a last_o / last_q stage shares its last unit with the next stage)
    end_unit = property(lambda self: self.first_unit + self.n_units - (1 if (self.last_o or self.last_q) else 0))

    def label(self) -> str:
        """e.g. '4m..8' = layer 4's MLP half through layer 8; '9..13a' ends with 13's attention
        half; '13m@6144..' / '..13a+6144': a gate/up boundary at column 6144 of layer 13;
        '13o..' / '..13q': an attention|o boundary in layer 13; '13k..' / '..13v': a
        q/k/v|attention boundary"""
        a = (f"{self.first_layer}{'m' if self.skip_first_attn else ''}{'o' if self.first_o else ''}"
             f"{'k' if self.first_q else ''}{f'@{self.first_col}' if self.first_col else ''}")
        b = (f"{self.last_layer}{'a' if self.skip_last_mlp else ''}{'q' if self.last_o else ''}"
             f"{'v' if self.last_q else ''}{f'+{self.last_col}' if self.last_col else ''}")
        return f"{a}..{b}"

    def span_kwargs(self) -> dict:
        """The SpanRuntime / PipelineStage keyword arguments of this range's boundaries."""
        return {"skip_first_attn": self.skip_first_attn, "skip_last_mlp": self.skip_last_mlp,
                "gateup_split_first": self.first_col, "gateup_split_last": self.last_col,
                "o_split_first": self.first_o, "o_split_last": self.last_o,
                "qkv_split_first": self.first_q, "qkv_split_last": self.last_q}

    def _key(self):
        return (self.first_unit, self.n_units, self.first_col, self.last_col, self.first_o, self.last_o,
                self.first_q, self.last_q)

    def __eq__(self, o):
        return isinstance(o, StageRange) and o._key() == self._key()

    def __repr__(self):
        return "StageRange({}, {}, {}, {}, {}, {}, {}, {})".format(*self._key())


def ranges_from_sizes(sizes) -> list:
    """Stage sizes in layers, multiples of one half (e.g. [4.5, 4.5, 5, ...]) -> StageRanges."""
    units = [int(round(2 * float(s))) for s in sizes]
    if any(u < 1 or abs(u - 2 * float(s)) > 1e-9 for u, s in zip(units, sizes)):
        raise ValueError(f"stage sizes must be positive multiples of 0.5 layers: {sizes}")
    return [StageRange(sum(units[:i]), u) for i, u in enumerate(units)]


def balanced_units(unit_costs, n: int, head_cost: float = 0.0, stage_cost: float = 0.0):
    """[StageRange] cutting the unit sequence (half layers, in order) into n contiguous stages
    minimising the slowest stage's cost -- each stage costs its units, plus stage_cost (its
    first RMSNorm launch) plus head_cost on the last stage -- ties to the smallest sum of
    squares.  Every stage gets at least one unit."""
    U = len(unit_costs)
    assert 1 <= n <= U
    pre = [0.0]
    for c in unit_costs:
        pre.append(pre[-1] + c)
    INF = (float("inf"), float("inf"))
    best = [[INF] * (U + 1) for _ in range(n + 1)]
    cut = [[0] * (U + 1) for _ in range(n + 1)]
    best[0][0] = (0.0, 0.0)
    for s in range(1, n + 1):
        for u in range(s, U - (n - s) + 1):
            for j in range(s - 1, u):
                mx, sq = best[s - 1][j]
                if mx == float("inf"):
                    continue
                c = pre[u] - pre[j] + stage_cost + (head_cost if s == n else 0.0)
                cand = (max(mx, c), sq + c * c)
                if cand < best[s][u]:
                    best[s][u], cut[s][u] = cand, j
    out, u = [], U
    for s in range(n, 0, -1):
        j = cut[s][u]
        out.append(StageRange(j, u - j))
        u = j
    return out[::-1]


# In-graph decode kernel means at Qwen3-8B, B = 16, ctx ~2.1k (rocprofv3 kernel trace of the
# round-4 decode graph, profiles/r04/decode_kernel_trace.json), us: the attention half
# (q/k/v GEMV + fused attention + o GEMV), the MLP half (gate/up + down GEMVs), a stage's first
# RMSNorm launch, and the last stage's final norm + lm_head GEMV + argmax.
DECODE_US_8B = {"attn_half": 12.70 + 26.88 + 8.73, "mlp_half": 33.57 + 19.99, "stage_norm": 5.19,
                "head": 5.19 + 201.5 + 4.24}


def halves_split(n_layers: int, n: int, costs: dict = DECODE_US_8B):
    """The half-layer split minimising the slowest stage's decode time (balanced_units over
    the measured per-half costs)."""
    units = [costs["attn_half"], costs["mlp_half"]] * n_layers
    return balanced_units(units, n, costs["head"], costs["stage_norm"])


# the gate/up share of the MLP half's decode time (profiles/r04/decode_kernel_trace.json:
# gate/up 33.57 us, down 19.99 us) -- what a column of the gate/up boundary costs
DECODE_US_8B_GATEUP = 33.57


# algorithmic decode bytes per unit at Qwen3-8B, B = 16, ctx 2k (bench.py kernel_bytes), MB: the
# attention half (norm, q/k/v, attention, o), the gate/up projection, the down projection, the
# last stage's final norm + lm_head
DECODE_MB_8B = {"attn_half": 221.6, "gateup": 202.2, "down": 101.6, "head": 1245.0, "o": 33.9, "qkv": 52.7}
# the o GEMV's and the (norm +) q/k/v GEMV's shares of the attention half
# (profiles/r04/decode_kernel_trace.json), us
DECODE_US_8B_O = 8.73
DECODE_US_8B_QKV = 12.70


def load_decode_costs(name: str = "qwen3_8b") -> dict:
    """The measured stage-boundary cost table (tools/boundary_costs.py on an MI355X, B = 16, ctx
    2048; profiles/r05/boundary_costs.json): us per decode-graph replay of small spans -- one
    layer, an attention half, an MLP half starting at each gate/up column, an attention half
    plus gate/up columns [0, c), the attention core, o + MLP, the head and the embedding."""
    import json
    import os
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", f"decode_costs_{name}.json")) as f:
        c = json.load(f)
    return apply_cost_fit(c)


def apply_cost_fit(c: dict) -> dict:
    """The cost table with its "projection_fit" (tools/fit_decode_costs.py: a least-squares fit
    of whole-stage measurements, bench.py --mode stages) applied: every table entry is a stage
    overhead plus content, content x content_scale, the overhead -> the fitted stage cost, the
    head x head_scale, and first_scale for the first stage (embedding, fed token ids)."""
    c = dict(c)
    for k in ("mlp", "send"):
        c[k] = {int(col): v for col, v in c[k].items()}
    fit = c.get("projection_fit")
    if fit:
        a, st0, st = fit["content_scale"], c["stage"], fit["stage"]
        for k in ("mlp", "send"):
            c[k] = {col: a * (v - st0) + st for col, v in c[k].items()}
        for k in ("attn", "core", "o_mlp", "one_layer", "q_send", "q_recv"):
            if k in c:
                c[k] = a * (c[k] - st0) + st
        c["layer"] *= a
        c["stage"] = st
        c["head"] *= fit["head_scale"]
        c["first_scale"] = fit["first_scale"]
    return c


def gateup_split(n_layers: int, n: int, intermediate: int, costs: dict = DECODE_US_8B, step: int = 256,
                 gateup_us: float = DECODE_US_8B_GATEUP, mb: dict = DECODE_MB_8B, o_cuts: bool = False,
                 o_us: float = DECODE_US_8B_O, cal: dict | None = None, q_cuts: bool = False,
                 q_us: float = DECODE_US_8B_QKV, vhead: dict | None = None):
    """Stages cut anywhere in the layer timeline a boundary may sit -- a layer start, or inside
    a layer's MLP before gate/up column c (c = 0: the half boundary; 0 < c < intermediate, a
    multiple of `step`: a gate/up boundary), and with o_cuts also between a layer's attention
    and its o projection -- so that the lowest stage's HBM fraction at the pipeline's tick,
    min_s bytes_s / max_s time_s, is the highest the time / byte model allows -- with q_cuts also
    between a layer's q/k/v projection and its attention (an exact search:
    for a tick bound T the best split is a DP over the cut points; T on a 4-us grid from the
    ideal total / n, then refined to 1 us).  Time model: costs (DECODE_US_8B) with the MLP
    half split into gate/up (gateup_us, linear in the columns) and down, and the attention half
    into its core and the o GEMV (o_us); bytes: mb.  Boundaries cannot sit inside the attention
    itself (its K/V live where it runs).

    cal (load_decode_costs(): measured stage times of small spans) replaces the time model: a
    stage costs cal["stage"] + its full layers x cal["layer"] + the part of the layer it starts
    in (o + MLP: cal["o_mlp"]; the MLP from gate/up column c: cal["mlp"][c]) + the part of the
    layer it ends in (the attention core: cal["core"]; the attention half + gate/up columns
    [0, c): cal["send"][c]) + head / embedding -- which prices what a boundary really costs
    (the partial gate/up GEMV's wave quantisation, the extra launches).

    vhead (the greedy head vocab-parallel, PipelineStage(sharded_head=True)): {"vocab", "row_mb"
    (one lm_head row, MB), "head_us" (the whole head's GEMV without the final norm), "fixed_us" (a
    shard's fixed cost), "norm_us" (the last stage's final norm), "step" (rows per shard step)}.
    The last stage then ends with the final norm, and every stage takes the lm_head rows that fill
    it up to the tick (water-filling, head_shard_split): for a tick T a stage's value is its bytes
    plus the rows (T - t - fixed) / per-row cost would stream, over T -- layer bytes that run slower
    than the head's GEMV are what a stage gives up to another; each candidate split is then priced
    with its real water-filled shards (every row placed once) and the best of those kept."""
    a, mlp, hd, sn = costs["attn_half"], costs["mlp_half"], costs["head"], costs["stage_norm"]
    ncol = intermediate // step
    emb, fs = 0.0, 1.0
    if cal is not None:
        fs = cal.get("first_scale", 1.0)
        assert all(k * step in cal["mlp"] and k * step in cal["send"] for k in range(ncol)), "cal: column grid"
        sn, hd, emb, lay = cal["stage"], cal["head"], cal["embed"], cal["layer"]
    # cut points in timeline order: (layer, kind, col) -- kind "L" a layer start, "O" before the
    # layer's o projection, "G" inside its MLP before gate/up column col * step; time and bytes
    # up to each cut.  A stage from cut j to cut l costs times[l] - times[j] + sadj[j] (the
    # receiving side's correction, cal) + sn (+ head, + embedding)
    cuts, times, byts, sadj, t, y = [], [], [], [], 0.0, 0.0
    for l in range(n_layers):
        cuts.append((l, "L", 0))
        times.append(t)
        byts.append(y)
        sadj.append(0.0)
        if q_cuts:
            cuts.append((l, "Q", 0))
            byts.append(y + mb["qkv"])
            if cal is None:
                times.append(t + q_us)
                sadj.append(0.0)
            else:
                times.append(t + cal["q_send"] - sn)
                sadj.append((cal["q_recv"] - sn) - (lay - (cal["q_send"] - sn)))
        if o_cuts:
            cuts.append((l, "O", 0))
            byts.append(y + mb["attn_half"] - mb["o"])
            if cal is None:
                times.append(t + a - o_us)
                sadj.append(0.0)
            else:
                times.append(t + cal["core"] - sn)
                sadj.append((cal["o_mlp"] - sn) - (lay - (cal["core"] - sn)))
        y += mb["attn_half"]
        for k in range(ncol):
            cuts.append((l, "G", k))
            byts.append(y + mb["gateup"] * k / ncol)
            if cal is None:
                times.append(t + a + gateup_us * k / ncol)
                sadj.append(0.0)
            else:
                te = cal["send"][k * step] - sn
                times.append(t + te)
                sadj.append((cal["mlp"][k * step] - sn) - (lay - te))
        t += (a + mlp) if cal is None else lay
        y += mb["gateup"] + mb["down"]
    cuts.append((n_layers, "L", 0))
    times.append(t)
    byts.append(y)
    sadj.append(0.0)
    # the search below needs cut times in order: measured send[c] is a staircase (wave
    # quantisation), made non-decreasing here (a flat step costs the same wherever it is cut)
    for i in range(1, len(times)):
        times[i] = max(times[i], times[i - 1])
    P = len(cuts) - 1

    # for a tick bound T: f[l] = the highest min over the stages so far of bytes / T with the
    # last of them ending at cut l and every stage within T (numpy over the previous cut j)
    import numpy as np
    tm, by, sa = np.array(times), np.array(byts), np.array(sadj)
    sa_lo = float(sa.min())
    # stages the engine refuses (inferd_span_create: a one-layer span cannot end before the part it
    # starts at; StageRange: no stage inside one attention unit, none without a whole unit): two cuts
    # of one layer where the first is the q/k/v|attention cut and the second the attention|o one, the
    # first the attention|o cut and the second inside the MLP, or both inside the MLP
    lay = np.array([c[0] for c in cuts])
    kq, ko, kg = (np.array([c[1] == k for c in cuts]) for k in ("Q", "O", "G"))

    if vhead is not None:
        per_row = vhead["head_us"] / vhead["vocab"]
        hd = vhead["norm_us"]                    # the last stage's own extra: the final norm
        mb = dict(mb, head=0.0)

    def stage_time(s, j, l):
        extra = sn + (hd if s == n - 1 else 0.0) + (emb if s == 0 else 0.0)
        return (tm[l] - tm[j] + sa[j] + extra) * (fs if s == 0 else 1.0)

    def real_value(b):
        """a split's lowest stage share at its tick with the shards water-filled (vhead)"""
        ts = [stage_time(s, b[s], b[s + 1]) for s in range(n)]
        rows = [r for _, r in head_shard_split(ts, vhead["vocab"], vhead["head_us"], vhead["fixed_us"],
                                               vhead["step"])]
        tick = max(t + (vhead["fixed_us"] + per_row * r if r else 0.0) for t, r in zip(ts, rows))
        return min(by[b[s + 1]] - by[b[s]] + rows[s] * vhead["row_mb"] for s in range(n)) / tick

    def solve(T):
        """(value, boundary cuts) of the best split with every stage within T (every end cut l of
        a stage at once: a [ends, window] matrix of its candidate start cuts j, ascending, so
        argmax keeps the first -- smallest -- best j)"""
        f = np.full(P + 1, -1.0)
        f[0] = np.inf
        arg = []
        for s in range(n):
            last = s == n - 1
            scale = fs if s == 0 else 1.0
            extra = sn + (hd if last else 0.0) + (emb if s == 0 else 0.0)
            g = np.full(P + 1, -1.0)
            gi = np.zeros(P + 1, dtype=np.int64)
            ends = np.array([P]) if last else np.arange(s + 1, P - (n - 1 - s) + 1)
            j0 = np.maximum(np.searchsorted(tm, tm[ends] - (T / scale - extra) + sa_lo, side="left"), s)
            W = int((ends - j0).max()) if len(ends) else 0
            if W > 0:
                J = j0[:, None] + np.arange(W)[None, :]
                valid = J < ends[:, None]
                Jc = np.where(valid, J, 0)
                e_ = ends[:, None]
                same = lay[Jc] == lay[e_]
                bad = same & ((kq[Jc] & ko[e_]) | (ko[Jc] & kg[e_]) | (kg[Jc] & kg[e_]))
                tst = (tm[ends][:, None] - tm[Jc] + sa[Jc] + extra) * scale
                ok = valid & ~bad & (tst <= T) & (f[Jc] >= 0)
                stage_mb = by[ends][:, None] - by[Jc] + (mb["head"] if last else 0.0)
                if vhead is not None:      # + the rows that fill the stage up to T
                    stage_mb = stage_mb + np.maximum(0.0, (T - tst - vhead["fixed_us"]) / per_row) * vhead["row_mb"]
                v = np.where(ok, np.minimum(f[Jc], stage_mb / T), -1.0)
                k = v.argmax(1)
                r = np.arange(len(ends))
                g[ends] = v[r, k]
                gi[ends] = Jc[r, k]
            arg.append(gi)
            f = g
        if f[P] < 0:
            return -1.0, None
        b, l = [P], P
        for s in range(n - 1, -1, -1):
            l = int(arg[s][l])
            b.append(l)
        return float(f[P]), b[::-1]
    # the tick: coarse grid from the ideal (total / n), then refined around the best
    lo_t = (times[P] + n * sn + hd + emb) / n
    if vhead is not None:     # the level every stage is filled to: the layers plus the whole head
        lo_t = (times[P] + n * sn + hd + emb + vhead["head_us"] + n * vhead["fixed_us"]) / n * 0.97
        _solve = solve

        def solve(T):       # noqa: F811 -- each T's split priced by its real water-filled shards
            v, bb = _solve(T)
            return (real_value(bb), bb) if bb is not None else (v, bb)
    best_val, best_b, best_T = -1.0, None, lo_t
    for T in np.arange(lo_t, lo_t * 1.08, 4.0):
        v, bb = solve(T)
        if v > best_val:
            best_val, best_b, best_T = v, bb, T
    T = lo_t * 1.08
    while best_b is None and T <= times[P] + n * sn + hd + emb + 4.0:
        # few layers per stage: no cover within 8 % of the ideal tick (the fixed stage costs weigh
        # more, whole units cannot be shared out); widen the bound until one exists
        T *= 1.02
        v, bb = solve(T)
        if v > best_val:
            best_val, best_b, best_T = v, bb, T
    for T in np.arange(best_T - 4.0, best_T + 4.0, 1.0):
        v, bb = solve(T)
        if v > best_val:
            best_val, best_b = v, bb
    b = best_b
    if b is None:
        raise ValueError(f"no split of {n_layers} layers into {n} stages the engine accepts")
    out = []
    for s in range(n):
        (l0, k0, c0), (l1, k1, c1) = cuts[b[s]], cuts[b[s + 1]]
        first_unit = 2 * l0 + (1 if k0 == "G" else 0)
        end_unit = 2 * l1 + (0 if k1 == "L" else 1)     # exclusive, in half units
        out.append(StageRange(first_unit, end_unit - first_unit, c0 * step if k0 == "G" else 0,
                              c1 * step if k1 == "G" else 0, k0 == "O", k1 == "O", k0 == "Q", k1 == "Q"))
    return out


def sublayer_split(n_layers: int, n: int, intermediate: int, **kw):
    """gateup_split with attention|o boundaries as cut points too."""
    return gateup_split(n_layers, n, intermediate, o_cuts=True, **kw)


def predicted_stage_us(r: StageRange, cal: dict, first: bool, last: bool) -> float:
    """A stage's decode-graph time on the measured cost table (load_decode_costs), us: the stage
    overhead, its full layers, the layer it starts in part-way (o + MLP, or the MLP from gate/up
    column first_col) and the one it ends in part-way (the attention core, or the attention half
    + gate/up columns [0, last_col)), head and embedding."""
    fs = cal.get("first_scale", 1.0) if first else 1.0
    t = cal["stage"] + (cal["embed"] if first else 0.0) + (cal["head"] if last else 0.0)
    l0, l1 = r.first_layer, r.last_layer
    start = cal["o_mlp"] - cal["stage"] if r.first_o else \
        cal["q_recv"] - cal["stage"] if r.first_q else \
        (cal["mlp"][r.first_col] - cal["stage"] if r.skip_first_attn else None)
    end = cal["core"] - cal["stage"] if r.last_o else \
        cal["q_send"] - cal["stage"] if r.last_q else \
        (cal["send"][r.last_col] - cal["stage"] if r.skip_last_mlp else None)
    if l0 == l1 and start is not None and end is not None:
        # one layer, cut on both sides: its start part less what its end part leaves out
        return fs * (t + start - (cal["layer"] - end))
    full = r.n_layers - (start is not None) - (end is not None)
    return fs * (t + full * cal["layer"] + (start or 0.0) + (end or 0.0))


def measured_split(n_layers: int, n: int, intermediate: int, o_cuts: bool = True, name: str = "qwen3_8b",
                   q_cuts: bool | None = None, **kw):
    """sublayer_split (or gateup_split) on the measured stage-boundary costs (load_decode_costs);
    q/k/v|attention cut points too (q_cuts, by default) where the table has their costs."""
    cal = load_decode_costs(name)
    if q_cuts is None:
        q_cuts = o_cuts and "q_send" in cal
    return gateup_split(n_layers, n, intermediate, o_cuts=o_cuts, cal=cal, q_cuts=q_cuts, **kw)


class SpanExecutor:
    """Runs one span's compute for pipeline items on this rank's GPU.  A decode item is one step of
    the microbatch's DecodeGraph: launched kernel by kernel (eager, the default: inferd_span_step,
    bit-identical to the replay and 6-8 us faster per stage step on the GPU, profiles/r05/
    stage_eager_ab.json) or as the captured graph's replay (eager=False)."""

    def __init__(self, span: SpanRuntime, eager: bool = True):
        self.span = span
        self.eager = eager
        self.device = span.device
        self.dims = span.dims
        self.has_embed, self.has_lm_head = span.has_embed, span.has_lm_head
        self.graphs = []

    def prefill(self, sessions, n_tokens, ids=None, x=None, want_ids=False, want_logits=False):
        """`sessions` each get n_tokens new tokens (ids on the first span, x otherwise).  Returns
        the hidden rows, or (last span) the greedy ids -- with want_logits (ids, last-row logits)."""
        out = self.span.forward([(sid, n_tokens) for sid in sessions], ids=ids, x=x,
                                want_hidden=not want_ids, want_next_ids=want_ids, want_logits=want_logits)
        if want_ids:
            return (out["next_ids"], out["logits"]) if want_logits else out["next_ids"]
        return out.get("record", out["hidden"])   # a decode-sized call across a gate/up boundary

    def prepare_decode(self, microbatches, n_steps, bufs):
        """Capture one decode graph per microbatch over its fixed buffers
        (bufs[m]: dict with ids / x / hidden_out / next_ids device tensors or None)."""
        self.graphs = [DecodeGraph(self.span, sessions, n_steps, **bufs[m])
                       for m, sessions in enumerate(microbatches)]

    def decode(self, m):
        if self.eager:
            self.graphs[m].launch_eager()
        else:
            self.graphs[m].launch()

    def head(self, normed, rows, keys_in=None, keys_out=None, ids=None):
        """This span's lm_head shard over `rows` normed rows (vocab-parallel head; SpanRuntime.head_shard)."""
        self.span.head_shard(normed, rows, keys_in, keys_out, ids)

    @staticmethod
    def combine(keys, n_parts, rows, ids):
        """ids from n_parts shards' keys [n_parts, rows] (torch.ops.inferd.argmax_combine)."""
        from .ops import ops as T
        T.argmax_combine(keys, n_parts, rows, ids)

    def profile_decode(self, microbatches, bufs, n_steps, head=None):
        """Eager (non-graph) decode steps with per-kernel-class HIP events on the launch
        stream, for kernel timings (HIP cannot time event-record nodes inside a replayed
        graph: hipEventElapsedTime rejects them); `head` (a callable) runs after every
        microbatch step (a vocab-parallel head's shard).  Returns {kernel class: (total ms, launches)}."""
        self.span.profile_start(1 << 17)
        for _ in range(n_steps):
            for m, sessions in enumerate(microbatches):
                states = [self.span.reserve(sid, 1) for sid in sessions]
                batch = self.span.build_batch([(st, 1) for st in states])
                b = bufs[m]
                self.span.run(batch, ids=b.get("ids"), x=b.get("x"), hidden=b.get("hidden_out"),
                              next_ids=b.get("next_ids"))
                if head is not None:
                    head()
                for st in states:
                    st.length += 1
        torch.cuda.synchronize(self.device)
        return self.span.profile_stop()


def ring_microbatches(world: int, sharded_head: bool = False, slack: int = 1) -> int:
    """Microbatches in flight on the decode ring: one per stage for the layer path, one per stage
    more when the greedy head runs vocab-parallel (its chain goes round the ring once more before the
    ids reach stage 0), plus `slack` (each unit lets the ring absorb one tick of summed hand-off
    latency: throughput = min(1 / tick, n_mb / (S * (tick + x))) per hop latency x)."""
    return world * (2 if sharded_head else 1) + (slack if world > 1 else 0)


def head_shard_split(stage_us, vocab: int, head_us: float, fixed_us: float = 6.0, step: int = 256,
                     min_rows: int = 0):
    """Rows of a vocab-parallel lm_head per stage ([(first, rows)] in stage order, covering
    [0, vocab)) that level the stages' decode times: stage s costs stage_us[s] (its layers) plus,
    with a shard of r rows, fixed_us + head_us * r / vocab (the shard GEMV streams r * hidden * 2
    bytes; fixed_us: its launches, ramp and key reduction).  Water-filling on a 0.01-us grid; rows in
    multiples of `step` (the remainder to the stage with the most room left).  min_rows: every stage
    gets at least that many rows (0: stages whose layers already reach the level get none)."""
    n = len(stage_us)
    per_row = head_us / vocab
    units = vocab // step
    assert units * step == vocab or vocab % 16 == 0

    def rows_at(level):
        return [max(0.0, (level - t - fixed_us) / per_row) for t in stage_us]
    lo, hi = min(stage_us), max(stage_us) + head_us + fixed_us
    for _ in range(100):
        mid = (lo + hi) / 2
        if sum(rows_at(mid)) >= vocab:
            hi = mid
        else:
            lo = mid
    want = rows_at(hi)
    rows = [max(min_rows, int(w // step) * step) for w in want]
    left = vocab - sum(rows)
    # hand out the rest in steps to the stages with the lowest resulting time
    while left > 0:
        cost = [stage_us[s] + (fixed_us + per_row * rows[s] if rows[s] else 0.0) for s in range(n)]
        s = min(range(n), key=lambda k: cost[k] + (fixed_us if rows[k] == 0 else 0.0))
        take = min(step, left)
        rows[s] += take
        left -= take
    while left < 0:      # min_rows overshoot: take back from the slowest
        cost = [stage_us[s] + fixed_us + per_row * rows[s] for s in range(n)]
        s = max((k for k in range(n) if rows[k] > min_rows), key=lambda k: cost[k])
        give = min(step, -left, rows[s] - min_rows)
        rows[s] -= give
        left += give
    out, f = [], 0
    for r in rows:
        out.append((f, r))
        f += r
    return out


class _InLink:
    """The receiving end of this stage's ring edge from its predecessor: the messages the predecessor
    sends, in its order (one communicator per edge keeps them FIFO), posted as receives a bounded
    window ahead of their use.  need() posts up to and including a message and makes the current
    stream wait for it (host-blocking only on gloo)."""

    def __init__(self, stage: "PipelineStage", msgs):
        self.st, self.msgs = stage, msgs
        self.index = {m: i for i, m in enumerate(msgs)}
        self.posted, self.high = 0, -1
        self.handles = {}

    def _post_next(self):
        spec = self.msgs[self.posted]
        self.handles[spec] = self.st._post_recv(spec)
        self.posted += 1

    def need(self, spec):
        """Receives are posted in the sender's order; they may be waited for in another order
        (with more slack than one item stage 0 uses a microbatch's ids after later normed rows)."""
        i = self.index[spec]
        self.high = max(self.high, i)
        while self.posted <= i:
            self._post_next()
        h, buf = self.handles.pop(spec)
        self.st._wait(h)
        return buf

    def drained(self) -> bool:
        return self.posted == len(self.msgs) and not self.handles

    def prefetch(self, n: int = 1):
        """keep the next n messages after the last one needed posted (their transfer overlaps the
        compute launched next)"""
        while self.posted < min(len(self.msgs), self.high + 1 + n):
            self._post_next()


class PipelineStage:
    """One rank of the span pipeline (rank 0 = FirstStage, rank S-1 = LastStage).

    Decode runs as an ASYNCHRONOUS RING (round 6): n_mb >= S microbatches are in flight and every
    stage processes work items (decode step k, microbatch m; item i = k * n_mb + m) in order, each as
    soon as its inputs have arrived -- there is no global tick.  Each directed ring edge s -> s+1 (and
    the wrap S-1 -> 0) is a 2-rank process group of its own, so every RCCL hand-off runs on that
    communicator's stream: a stage posts the receive of item i+1 before it launches item i (the
    transfer overlaps the compute), its sends are posted right after the producing launch, and the
    compute stream waits (work.wait(): a stream wait, the host never blocks on RCCL) only on the
    input it is about to use.  With n_mb = S + 1 the ring holds one item of slack: throughput is
    min(1 / c, n_mb / (S (c + x))) for stage time c and per-hop latency x, so up to x = c / S of
    hand-off per hop is hidden.

    Vocab-parallel greedy head (sharded_head): the last stage ends with the final norm and hands the
    normed last rows (128 KiB at B = 16) round the ring; stage s runs its lm_head shard on them S
    items after the layers (one ring lap behind), folding its (max logit, first index) keys into the
    running keys it forwards; the last stage's shard finishes the argmax and sends the ids to stage
    0.  Every hand-off stays on the ring's own edges (one inbound and one outbound communicator per
    GPU).  Item j's ids reach stage 0 S iterations after its normed rows left the last stage, 2S
    iterations after stage 0 ran its layers: n_mb = 2S + slack."""

    def __init__(self, dims: ModelDims, rank: int, world: int, first_layer: int, n_layers: int, *,
                 device, seed: int, n_microbatches: int, batch: int, max_ctx: int, prefill_chunk: int = 2,
                 executor=None, group=None, profile: str = "random", want_logits: bool = False,
                 skip_first_attn: bool = False, skip_last_mlp: bool = False, gateup_split_first: int = 0,
                 gateup_split_last: int = 0, o_split_first: bool = False, o_split_last: bool = False,
                 qkv_split_first: bool = False, qkv_split_last: bool = False, eager_decode: bool = True,
                 sharded_head: bool = False, head_shard=(0, 0)):
        """profile: the synthetic weight profile (runtime.SpanRuntime.init_synthetic: "peaked"
        for token-exact parity runs).  want_logits (last stage, whole head only): every decode step's
        and the prefill's last-row logits are kept, for parity checks against the oracle's.
        skip_first_attn / skip_last_mlp / gateup_split_* / o_split_* / qkv_split_*: the stage's
        sub-layer boundaries (StageRange.span_kwargs(); the hand-offs are records, handoff_elems).
        n_microbatches: >= world (ring_microbatches(world, sharded_head) adds the ring's slack).
        sharded_head / head_shard: the greedy head vocab-parallel over the stages, this stage owning
        lm_head rows [head_shard[0], head_shard[0] + head_shard[1]) -- the shards in stage order,
        contiguous from row 0 (head_shard_split)."""
        assert n_microbatches >= world * (2 if sharded_head and world > 1 else 1), \
            "the ring needs a microbatch per stage in flight (two with a vocab-parallel head)"
        assert not (sharded_head and want_logits), "logits capture needs the whole head on the last stage"
        self.dims, self.rank, self.world = dims, rank, world
        self.S = world
        self.n_mb, self.B = n_microbatches, batch
        self.device = torch.device(device)
        self.group = group
        self.prefill_chunk = prefill_chunk
        self.sharded = bool(sharded_head) and world > 1
        self.head_first, self.head_rows = (int(head_shard[0]), int(head_shard[1])) if self.sharded else (0, 0)
        last = rank == world - 1
        if executor is None:
            pages_per_seq = (max_ctx + KV_PAGE - 1) // KV_PAGE + 1
            span = SpanRuntime(dims, first_layer, n_layers, has_embed=(rank == 0), has_lm_head=last and not self.sharded,
                               kv_pages=n_microbatches * batch * pages_per_seq + 4,
                               max_tokens=max(prefill_chunk * max_ctx, batch), max_seqs=max(batch, prefill_chunk),
                               max_positions=max_ctx, device=self.device, skip_first_attn=skip_first_attn,
                               skip_last_mlp=skip_last_mlp, gateup_split_first=gateup_split_first,
                               gateup_split_last=gateup_split_last, o_split_first=o_split_first,
                               o_split_last=o_split_last, qkv_split_first=qkv_split_first,
                               qkv_split_last=qkv_split_last, head_first=self.head_first, head_rows=self.head_rows,
                               final_norm_out=last and self.sharded)
            span.init_synthetic(seed, profile)
            executor = SpanExecutor(span, eager=eager_decode)
        self.ex = executor
        self.span = getattr(executor, "span", None)
        self.sessions = [[("mb", m, b) for b in range(batch)] for m in range(n_microbatches)]
        h = dims.hidden
        dev = self.device
        mb = range(n_microbatches)
        self.col_in, self.col_out = gateup_split_first, gateup_split_last
        self.o_in, self.o_out = bool(o_split_first), bool(o_split_last)
        self.q_in, self.q_out = bool(qkv_split_first), bool(qkv_split_last)

        def buf(col, o, q):     # a decode hand-off buffer: a record (1-D) or [batch, hidden]
            if col or o or q:
                return torch.zeros(buffer_elems(dims, batch, col, o, True, q), dtype=torch.bfloat16, device=dev)
            return torch.zeros(batch, h, dtype=torch.bfloat16, device=dev)
        self.ids = [torch.zeros(batch, dtype=torch.int32, device=dev) for _ in mb]
        self.h_in = [buf(self.col_in, self.o_in, self.q_in) for _ in mb]
        self.h_out = [buf(self.col_out, self.o_out, self.q_out) for _ in mb]
        self.ids_out = [torch.zeros(batch, dtype=torch.int32, device=dev) for _ in mb]
        # vocab-parallel head: the last stage's final-normed rows (fragment-packed 16-row tiles) and
        # every stage's head record [normed rows | running keys int64 [B]] (bytes)
        self.normed_bytes = (batch + 15) // 16 * 16 * h * 2
        if self.sharded:
            self.normed = [torch.zeros(self.normed_bytes // 2, dtype=torch.bfloat16, device=dev) for _ in mb] \
                if last else None
            self.head_rec = [torch.zeros(self.normed_bytes + 8 * batch, dtype=torch.uint8, device=dev) for _ in mb]
        self.want_logits = want_logits and last
        self.logits = [torch.zeros(batch, dims.vocab, dtype=torch.bfloat16, device=dev) for _ in mb] \
            if self.want_logits else None
        self.step_base = 0   # decode steps already run (absolute step of the next decode call)
        # host time per tick of the last decode() call, split into the hand-off (posts and waits)
        # and the rest (launches, page-table advance, schedule bookkeeping)
        self.tick_stats = None
        self.first_layer, self.n_layers = first_layer, n_layers
        self._exchanged = False     # first hand-off done (logged once)
        self._inflight = None       # the last exchange's transient tensors (see _exchange)
        self._pending = {}          # buffer key -> a send still reading that buffer
        self.prev_rank, self.next_rank = (rank - 1) % world, (rank + 1) % world
        self.link_in = self.link_out = None
        # streams (GPU ranks of a multi-stage pipeline): every launch of the stage runs on a compute
        # stream with a hardware queue of its own (torch.ops.inferd.dedicated_stream), so an RCCL
        # receive posted ahead of its data -- resident on its communicator's stream -- never holds
        # back a compute kernel that happens to share its queue; receives are posted from a side
        # stream that waits only on the event of the buffer's last use (self._use), not on the
        # compute queued since
        self.cstream = self.pstream = None
        self._use = {}
        if world > 1 and self.device.type == "cuda":
            from .ops import ops as T
            self.cstream = torch.cuda.ExternalStream(T.dedicated_stream(self.device), device=self.device)
            self.pstream = torch.cuda.Stream(device=self.device)
        if world > 1:
            with self._compute():
                self._make_links()

    @property
    def first(self):
        return self.rank == 0

    @property
    def last(self):
        return self.rank == self.S - 1

    def head_normed(self, rec):
        return rec[:self.normed_bytes].view(torch.bfloat16)

    def head_keys(self, rec):
        return rec[self.normed_bytes:self.normed_bytes + 8 * self.B].view(torch.int64)

    # ------------------------------------------------------------------ ring links
    def _global(self, r: int) -> int:
        import torch.distributed as dist
        return r if self.group is None else dist.get_global_rank(self.group, r)

    def _make_links(self):
        """One 2-rank process group per directed ring edge e -> e+1 (e = 0 .. S-1; at S = 2 the two
        directions are two groups over the same pair), created by every rank in the same order (as
        new_group requires), then warmed up edge by edge in that order: RCCL sets a p2p connection up
        at its first use, so each edge's first send / receive happens here, pairwise in a global
        order -- no rank can be waiting on a connection its partner has not reached."""
        import torch.distributed as dist
        S = self.S
        links = [dist.new_group([self._global(e), self._global((e + 1) % S)]) for e in range(S)]
        self.link_out, self.link_in = links[self.rank], links[(self.rank - 1) % S]
        one = torch.zeros(1, dtype=torch.int32, device=self.device)
        for e in range(S):
            if self.rank == e:
                self._wait(self._post(True, one, (e + 1) % S, links[e]))
            elif self.rank == (e + 1) % S:
                self._wait(self._post(False, one, e, links[e]))
        if self.device.type == "cuda":
            torch.cuda.current_stream(self.device).synchronize()

    def _post(self, send: bool, t, peer: int, group):
        """Post one isend / irecv of tensor t to / from stage `peer` on `group`.  Returns a handle
        for _wait.  RCCL: the op runs on the group's stream after the current stream's earlier
        work.  gloo with device tensors (GPU ranks rehearsing without RCCL): staged through host
        memory (a send copies out at once; a receive lands in a host tensor copied in at _wait)."""
        import torch.distributed as dist
        staged = t.is_cuda and dist.get_backend(group) == "gloo"
        dst = None
        if staged:
            if send:
                t = t.cpu()
            else:
                dst, t = t, torch.empty(t.shape, dtype=t.dtype)
        works = dist.batch_isend_irecv([dist.P2POp(dist.isend if send else dist.irecv, t, self._global(peer), group)])
        return works, t, dst

    @staticmethod
    def _wait(h):
        works, t, dst = h
        for w in works:
            w.wait()
        if dst is not None:
            dst.copy_(t)

    def _settle(self, key):
        """Before a buffer is written again (by a launch or a receive): the send still reading it
        must be done -- on RCCL a stream wait (free: the send was posted an item or more ago)."""
        h = self._pending.pop(key, None)
        if h is not None:
            self._wait(h)

    def _send(self, key, t):
        self._settle(key)
        self._pending[key] = self._post(True, t, self.next_rank, self.link_out)

    def _used(self, *keys):
        """The compute stream's launches so far are the last users of these buffers (an event per
        buffer; a receive into one waits on it, _post_recv)."""
        if self.cstream is None:
            return
        for k in keys:
            ev = self._use.get(k)
            if ev is None:
                ev = self._use[k] = torch.cuda.Event()
            ev.record(self.cstream)

    def _post_recv(self, spec):
        """Post the receive of ring message `spec` into its buffer, once the buffer's last user (a
        launch, _used; a send forwarding it, _pending) is done -- from the side stream, so the receive
        starts then and not after the compute queued since.  Returns (handle, buffer)."""
        buf, key = self._recv_buf(spec)
        if self.pstream is None:
            self._settle(key)
            return self._post(False, buf, self.prev_rank, self.link_in), buf
        with torch.cuda.stream(self.pstream):
            self._settle(key)                       # a forwarded record still being sent from it
            ev = self._use.get(key)
            if ev is not None:
                self.pstream.wait_event(ev)
            return self._post(False, buf, self.prev_rank, self.link_in), buf

    def _compute(self):
        """Context: the stage's launches on its compute stream, ordered after the caller's stream's
        earlier work and before its later work."""
        import contextlib
        if self.cstream is None:
            return contextlib.nullcontext()
        st = self

        class _Ctx:
            def __enter__(self):
                self.caller = torch.cuda.current_stream(st.device)
                st.cstream.wait_stream(self.caller)
                self.cm = torch.cuda.stream(st.cstream)
                self.cm.__enter__()

            def __exit__(self, *a):
                self.cm.__exit__(*a)
                self.caller.wait_stream(st.cstream)
        return _Ctx()

    # messages on the edge out of stage s at iteration t of a decode call of n items (the sender's
    # order; one communicator per edge keeps them FIFO): ("h", i) the layer hand-off of item i,
    # ("k", j) the head record after stage s's shard of item j, ("n", t) the last stage's normed rows,
    # ("i", j) the greedy ids of item j (last stage -> stage 0)
    def _msgs_out(self, s: int, t: int, n_items: int, D: int):
        last = s == self.S - 1
        out = []
        if t < n_items:
            out.append(("h", t) if not last else (("n", t) if self.sharded else ("i", t)))
        j = t - D
        if self.sharded and 0 <= j < n_items:
            out.append(("i", j) if last else ("k", j))
        return out

    def _recv_buf(self, spec):
        """(tensor, buffer key) a message lands in on this stage"""
        kind, i = spec
        m = i % self.n_mb
        if kind == "h":
            t = self.h_in[m]
            if self.col_in or self.o_in or self.q_in:
                t = t[:handoff_elems(self.dims, self.B, self.col_in, self.o_in, True, self.q_in)]
            return t, ("h_in", m)
        if kind == "i":
            return self.ids[m], ("ids", m)
        if kind == "n":
            return self.head_normed(self.head_rec[m]), ("head", m)
        return self.head_rec[m], ("head", m)

    def _bufs(self, m):
        """Fixed buffers of microbatch m for this stage's role."""
        lg = {"logits": self.logits[m]} if self.want_logits else {}
        if self.S == 1:
            return {"ids": self.ids[m], "x": None, "hidden_out": None, "next_ids": self.ids[m], **lg}
        if self.first:
            return {"ids": self.ids[m], "x": None, "hidden_out": self.h_out[m], "next_ids": None}
        if self.last:
            if self.sharded:
                return {"ids": None, "x": self.h_in[m], "hidden_out": self.normed[m], "next_ids": None}
            return {"ids": None, "x": self.h_in[m], "hidden_out": None, "next_ids": self.ids_out[m], **lg}
        return {"ids": None, "x": self.h_in[m], "hidden_out": self.h_out[m], "next_ids": None}

    def _exchange(self, send=None, send_to=None, recv=None, recv_from=None):
        """One grouped hand-off on the pipeline's process group (prefill; lockstep): isend `send`
        to stage send_to, irecv `recv` from stage recv_from (the reference's HTTP hop
        node.py:102-130, as RCCL p2p over xGMI).

        Tensor lifetimes on the nccl path (RCCL runs on its own stream; `work.wait()` makes
        torch's current stream wait for it without blocking the host, and the process group
        orders its stream after the current stream's earlier work): the prefill send is a per-chunk
        output and the recv a fresh tensor per tick; both are kept referenced here until the NEXT
        exchange, so the caching allocator cannot hand their blocks to a new tensor while the send
        may be in flight, whether or not the process group records its stream on p2p inputs; the
        first-ids hand-off after prefill (`flat`) likewise.  On gloo (CPU-rank tests, GPU ranks
        rehearsing without RCCL) device tensors are staged through host memory synchronously."""
        import torch.distributed as dist
        staged = dist.get_backend(self.group) == "gloo"
        dst = None
        if staged:
            if send is not None and send.is_cuda:
                send = send.cpu()
            if recv is not None and recv.is_cuda:
                dst, recv = recv, torch.empty(recv.shape, dtype=recv.dtype)
        ops = []
        if send is not None:
            ops.append(dist.P2POp(dist.isend, send, self._global(send_to), self.group))
        if recv is not None:
            ops.append(dist.P2POp(dist.irecv, recv, self._global(recv_from), self.group))
        t0 = time.perf_counter() if not self._exchanged else 0.0
        if ops:
            for w in dist.batch_isend_irecv(ops):
                w.wait()
        if dst is not None:
            dst.copy_(recv)
        self._inflight = (send, recv)     # released at the next exchange (lifetimes above)
        if not self._exchanged and ops:
            # first hand-off of this stage: confirm it completed, so a wedged p2p link names
            # itself (with the process group's timeout) instead of hanging silently
            self._exchanged = True
            if self.device.type == "cuda":
                torch.cuda.current_stream(self.device).synchronize()
            print(f"[pipeline] rank {self.rank}/{self.S} ({self.device}, layers {self.first_layer}.."
                  f"{self.first_layer + self.n_layers - 1}): first exchange done over {dist.get_backend(self.group)}"
                  f" (send->{send_to if send is not None else '-'}, recv<-{recv_from if recv is not None else '-'},"
                  f" {(time.perf_counter() - t0) * 1e3:.1f} ms)", file=sys.stderr, flush=True)

    # ------------------------------------------------------------------ head (vocab-parallel)
    def _head(self, normed, keys_in, keys_out, ids):
        """This stage's lm_head shard over the B normed rows, folded into the running keys (or the
        ids on the last stage).  Shards run in stage order from row 0 (head_shard_split), so the
        running keys are live iff an earlier stage owns rows (head_first > 0): the first stage with
        rows starts them, a stage without rows passes the record on untouched."""
        live = self.head_first > 0
        if self.head_rows:
            self.ex.head(normed, self.B, keys_in=keys_in if live else None, keys_out=keys_out, ids=ids)
        elif ids is not None:
            self.ex.combine(keys_in, 1, self.B, ids)

    # ------------------------------------------------------------------ prefill
    @torch.no_grad()
    def prefill(self, prompts, capture=None):
        with self._compute():
            self._prefill(prompts, capture)

    def _prefill(self, prompts, capture=None):
        """prompts: per microbatch an int tensor [B, T] (read on the first stage only).
        Runs every microbatch's prompt through the pipeline in chunks of prefill_chunk
        sequences; leaves the first decode ids of every microbatch on stage 0.  `capture`
        (a dict): on non-last stages it receives this stage's output for the first chunk of
        microbatch 0 -- its sequences 0 .. prefill_chunk-1, [chunk * T, h] -- as a CPU copy
        (the stage-boundary hidden state parity tests compare with the oracle); on the last
        stage of a want_logits pipeline, capture["logits"][m] = microbatch m's last-row logits
        [B, vocab] (CPU)."""
        S, T = self.S, prompts[0].shape[1]
        items = [(m, c) for m in range(self.n_mb) for c in range(0, self.B, self.prefill_chunk)]
        h = self.dims.hidden
        first_ids = [None] * self.n_mb
        ids_parts = {}
        bufs_in, bufs_out = {}, {}
        for t in range(len(items) + S):
            i_send = t - 1 - self.rank          # item produced last tick
            i_cur = t - self.rank               # item computed this tick
            send = recv = None
            if not self.last and 0 <= i_send < len(items):
                send = bufs_out.pop(i_send)
                m, c = items[i_send]
                rows = min(self.prefill_chunk, self.B - c) * T
                if (self.col_out and rows <= 64) or self.o_out or (self.q_out and T == 1):     # a record hand-off
                    send = send.reshape(-1)[:handoff_elems(self.dims, rows, self.col_out, self.o_out, T == 1,
                                                           self.q_out)]
            if not self.first and 0 <= i_cur < len(items):
                m, c = items[i_cur]
                nseq = min(self.prefill_chunk, self.B - c)
                rows = nseq * T
                if (self.col_in and rows <= 64) or self.o_in or (self.q_in and T == 1):
                    recv = torch.zeros(buffer_elems(self.dims, rows, self.col_in, self.o_in, T == 1, self.q_in),
                                       dtype=torch.bfloat16, device=self.device)
                    bufs_in[i_cur] = recv
                    recv = recv[:handoff_elems(self.dims, rows, self.col_in, self.o_in, T == 1, self.q_in)]
                else:
                    recv = torch.empty(rows, h, dtype=torch.bfloat16, device=self.device)
                    bufs_in[i_cur] = recv
            if S > 1:
                self._exchange(send, (self.rank + 1) % S, recv, (self.rank - 1) % S)
            if 0 <= i_cur < len(items):
                m, c = items[i_cur]
                sess = self.sessions[m][c:c + self.prefill_chunk]
                wl = self.want_logits and capture is not None
                kw = {"want_logits": True} if wl else {}
                want_ids = self.last and not self.sharded
                if self.first:
                    ids = prompts[m][c:c + len(sess)].reshape(-1).to(self.device, torch.int32)
                    out = self.ex.prefill(sess, T, ids=ids, want_ids=want_ids, **kw)
                else:
                    out = self.ex.prefill(sess, T, x=bufs_in.pop(i_cur), want_ids=want_ids, **kw)
                if self.last:
                    if wl:
                        out, lg = out
                        capture.setdefault("logits_parts", {})[(m, c)] = lg.cpu()
                    ids_parts[(m, c)] = out      # the greedy ids, or (vocab-parallel head) the normed rows
                else:
                    bufs_out[i_cur] = out
                    if capture is not None and i_cur == 0:     # h1 rows (the head of a record)
                        capture["hidden"] = out.reshape(-1)[:len(sess) * T * h].reshape(len(sess) * T, h).cpu()
        if self.sharded:
            self._prefill_head(ids_parts)
            return
        if self.last:
            for m in range(self.n_mb):
                first_ids[m] = torch.cat([ids_parts[(m, c)] for c in range(0, self.B, self.prefill_chunk)])
            if capture is not None and "logits_parts" in capture:
                parts = capture.pop("logits_parts")
                capture["logits"] = [torch.cat([parts[(m, c)] for c in range(0, self.B, self.prefill_chunk)])
                                     for m in range(self.n_mb)]
        # hand the first decode ids to stage 0
        if S == 1:
            for m in range(self.n_mb):
                self.ids[m].copy_(first_ids[m])
        else:
            flat = torch.empty(self.n_mb * self.B, dtype=torch.int32, device=self.device)
            if self.last:
                flat.copy_(torch.cat(first_ids))
                self._exchange(send=flat, send_to=0)
            elif self.first:
                self._exchange(recv=flat, recv_from=S - 1)
                for m in range(self.n_mb):
                    self.ids[m].copy_(flat[m * self.B:(m + 1) * self.B])

    def _prefill_head(self, normed_parts):
        """The vocab-parallel head of every microbatch's prompt (its last rows): the last stage's
        normed rows go to stage 0 and along the ring through every shard, the last stage finishes
        the argmax and returns the first decode ids to stage 0 -- one microbatch at a time on the
        pipeline's group (untimed)."""
        S, h, B = self.S, self.dims.hidden, self.B
        full = {}
        if self.last:     # each chunk's packed rows -> the microbatch's B rows, packed
            for m in range(self.n_mb):
                rows = [unpack_rows(normed_parts[(m, c)].reshape(-1), min(self.prefill_chunk, B - c), h)
                        for c in range(0, B, self.prefill_chunk)]
                full[m] = torch.zeros(self.normed_bytes // 2, dtype=torch.bfloat16, device=self.device)
                p = pack_rows(torch.cat(rows))
                full[m][:p.numel()].copy_(p)
        for m in range(self.n_mb):
            rec = self.head_rec[m]
            if self.last:
                self._exchange(send=full[m], send_to=0)
                self._exchange(recv=rec, recv_from=S - 2)
                self._head(full[m], self.head_keys(rec), None, self.ids_out[m])
                self._exchange(send=self.ids_out[m], send_to=0)
                continue
            if self.first:
                self._exchange(recv=self.head_normed(rec), recv_from=S - 1)
                self._head(self.head_normed(rec), None, self.head_keys(rec), None)
            else:
                self._exchange(recv=rec, recv_from=self.rank - 1)
                self._head(self.head_normed(rec), self.head_keys(rec), self.head_keys(rec), None)
            self._exchange(send=rec, send_to=self.rank + 1)
            if self.first:
                self._exchange(recv=self.ids[m], recv_from=S - 1)
        self._inflight = (full, None)
        if self.device.type == "cuda":
            torch.cuda.current_stream(self.device).synchronize()

    # ------------------------------------------------------------------ decode
    def prepare_decode(self, n_steps: int):
        """Reserve cache pages for n_steps tokens per sequence and capture the decode graphs."""
        with self._compute():
            self.ex.prepare_decode(self.sessions, n_steps, [self._bufs(m) for m in range(self.n_mb)])

    @torch.no_grad()
    def decode(self, n_steps: int, record=None, record_logits=None, force=None):
        with self._compute():
            self._decode(n_steps, record, record_logits, force)

    def _decode(self, n_steps: int, record=None, record_logits=None, force=None):
        """Run n_steps decode steps of every microbatch.  `record` (stage 0 only): list that
        receives (absolute step, microbatch, ids tensor copy) of every input fed to the first
        span; `record_logits` (last stage of a want_logits pipeline): list that receives
        (absolute step, microbatch, device copy of the step's last-row logits [B, vocab]);
        `force` (stage 0 only, teacher forcing for parity runs): int tensor [steps, B] -- the
        ids fed at absolute step k are force[k] instead of the last stage's greedy choice.
        Sets self.tick_stats: host microseconds per item, hand-off (posts and waits) and the rest.
        On return stage 0 holds every microbatch's next ids (the next call continues the ring)."""
        def feed(k, m):
            if force is not None and self.first:
                self.ids[m].copy_(force[self.step_base + k].to(self.ids[m].device, torch.int32),
                                  non_blocking=True)
        S, n_mb = self.S, self.n_mb
        n_items = n_steps * n_mb
        t_x = 0.0
        t0 = time.perf_counter()
        if S == 1:
            for i in range(n_items):
                k, m = divmod(i, n_mb)
                feed(k, m)
                if record is not None:
                    record.append((self.step_base + k, m, self.ids[m].clone()))
                self.ex.decode(m)
                if record_logits is not None and self.want_logits:
                    record_logits.append((self.step_base + k, m, self.logits[m].clone()))
            self.step_base += n_steps
            self._tick_stats(n_items, time.perf_counter() - t0, 0.0)
            return
        D = S if self.sharded else 0          # the head runs one ring lap behind the layers
        n_iter = n_items + D
        pred = (self.rank - 1) % S
        link = _InLink(self, [m for t in range(n_iter) for m in self._msgs_out(pred, t, n_items, D)])
        hand = self.col_out or self.o_out or self.q_out
        n_hand = handoff_elems(self.dims, self.B, self.col_out, self.o_out, True, self.q_out) if hand else 0
        for it in range(n_iter):
            if it < n_items:
                k, m = divmod(it, n_mb)
                tx = time.perf_counter()
                if not self.first:
                    link.need(("h", it))
                elif it >= n_mb:
                    link.need(("i", it - n_mb))       # this microbatch's ids, from its previous step
                t_x += time.perf_counter() - tx
                feed(k, m)
                if self.first and record is not None:
                    record.append((self.step_base + k, m, self.ids[m].clone()))
                out_key, out = (("h_out", m), self.h_out[m]) if not self.last else \
                    ((("normed", m), self.normed[m]) if self.sharded else (("ids_out", m), self.ids_out[m]))
                self._settle(out_key)
                self.ex.decode(m)
                self._used(("ids", m) if self.first else ("h_in", m))
                if record_logits is not None and self.want_logits:
                    record_logits.append((self.step_base + k, m, self.logits[m].clone()))
                tx = time.perf_counter()
                self._send(out_key, out[:n_hand] if (hand and not self.last) else out)
                # the next message's receive, posted after this iteration's sends: a receive waiting
                # for its data never sits in front of a send (two communicators may share a queue)
                link.prefetch(1)
                t_x += time.perf_counter() - tx
            j = it - D
            if self.sharded and 0 <= j < n_items:
                mj = j % n_mb
                tx = time.perf_counter()
                link.need(("n", j) if self.first else ("k", j))     # lands in head_rec[mj]
                t_x += time.perf_counter() - tx
                rec = self.head_rec[mj]
                if self.last:
                    self._settle(("ids_out", mj))
                    self._head(self.normed[mj], self.head_keys(rec), None, self.ids_out[mj])
                    self._used(("head", mj))
                    tx = time.perf_counter()
                    self._send(("ids_out", mj), self.ids_out[mj])
                else:
                    self._head(self.head_normed(rec), None if self.first else self.head_keys(rec),
                               self.head_keys(rec), None)
                    self._used(("head", mj))
                    tx = time.perf_counter()
                    self._send(("head", mj), rec)
                link.prefetch(1)
                t_x += time.perf_counter() - tx
        if self.first:     # the next call's first ids: the last n_mb items' greedy choices
            tx = time.perf_counter()
            for j in range(max(0, n_items - n_mb), n_items):
                link.need(("i", j))
            t_x += time.perf_counter() - tx
        assert link.drained(), "decode ended with ring messages not received"
        for key in list(self._pending):
            self._settle(key)
        self.step_base += n_steps
        self._tick_stats(n_iter, time.perf_counter() - t0, t_x)

    def _tick_stats(self, ticks, total_s, exchange_s):
        self.tick_stats = {"ticks": ticks, "host_us_per_tick": round((total_s - exchange_s) / ticks * 1e6, 1),
                           "exchange_us_per_tick": round(exchange_s / ticks * 1e6, 1)}

    def profile_decode(self, n_steps: int):
        """Per-kernel timings from eager (event-instrumented) decode steps on this stage,
        without exchanges (kernel durations do not depend on where inputs came from); with a
        vocab-parallel head each step also runs this stage's shard."""
        head = None
        if self.sharded:
            rec = self.head_rec[0]
            normed = self.normed[0] if self.last else self.head_normed(rec)
            head = lambda: self._head(normed, self.head_keys(rec) if not self.first else None,  # noqa: E731
                                      None if self.last else self.head_keys(rec),
                                      self.ids_out[0] if self.last else None)
        with self._compute():
            return self.ex.profile_decode(self.sessions, [self._bufs(m) for m in range(self.n_mb)], n_steps, head)

    def release(self):
        if self.span is not None:
            self.ex.graphs = []
            self.span.release_all()
