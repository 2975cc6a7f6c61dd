"""One petals node served by a group of GPUs: the node API on rank 0, the stage's layers split
over every rank of a torch.distributed group, hidden rows handed rank -> rank.

The reference gives one node one span (`petals/node.py:47-50` builds one PartitionedQwen2 per
process).  Inside one 8-GPU host a stage's layers can be spread over several GPUs and still
register in the DHT as ONE node: rank 0 of the group runs the unchanged aiohttp node and this
class as its `PartitionedQwen2`; ranks 1.. run `serve_forever()`.

    # every rank (torchrun --nproc-per-node N ...):
    grp = SpanGroup(model_name, num_stages, stage, parts_path)     # same args as the reference
    if grp.rank == 0:  run the node with grp as its model (node.py:47-50)
    else:              grp.serve_forever()

Per request rank 0 broadcasts a small header (the requests' session keys and row counts), runs
its sub-span, and each rank passes its output rows to the next (RCCL send/recv on the `nccl`
backend; host-staged on gloo); the group's last rank returns the hidden rows or, on the
chain's last stage, the greedy ids to rank 0, which answers with the reference's output
schema.  Sessions (PartitionedQwen2's optional session_id) live on every rank with identical
page accounting: rank 0 reserves and evicts first, then tells the others.

Faults keep the group in lockstep.  Rank 0 validates a request (shapes, token ids) before it
broadcasts anything, so a malformed request never reaches the other ranks.  Every hand-off
carries a status word ahead of its rows: a rank whose compute raises (or whose predecessor
failed) forwards zero rows with the failing rank's status and message instead of leaving its
successor blocked; rank 0 then drops the request's sessions on every rank and raises the
failing rank's error, and every rank keeps serving.
Layer split inside the group: pipeline.balanced_split (the lm_head priced on the rank that
owns it, in decode bytes) over the stage's [start_layer, end_layer].

A SpanGroup adds CAPACITY (a stage too large for one GPU's memory, KV pages for more sessions),
not throughput: the reference's node serves one request at a time (task_scheduler.py:18), so a
request walks the group's ranks one after another and N GPUs each run 1/N of the time.  The
throughput of N GPUs is the RCCL pipeline of inferd_amd/pipeline.py (N microbatches in flight).
"""
from __future__ import annotations

import json
import os
from collections import OrderedDict

import torch

from .partitioned_models import (_BF16, PartitionedQwen2, _load_tokenizer, _make_stage, _model_key,
                                 _span_kwargs)
from .runtime import MODELS, ModelDims, SpanRuntime


def stage_range(parts_path: str, model_name: str, num_stages: int, stage: int):
    """(dims, start_layer, end_layer, profile or None) of a stage spec or stage file."""
    if parts_path.startswith("synthetic:"):
        bits = parts_path.split(":")
        dims = MODELS[bits[2] if len(bits) > 2 and bits[2] else _model_key(model_name)]
        if len(bits) > 4:
            start, end = int(bits[3]), int(bits[4])
        else:
            per = dims.layers // num_stages
            start = stage * per
            end = dims.layers - 1 if stage == num_stages - 1 else start + per - 1
        return dims, start, end, (bits[5] if len(bits) > 5 else "random")
    from safetensors import safe_open
    with safe_open(parts_path, framework="pt", device="cpu") as f:
        meta = f.metadata()
    return ModelDims(**json.loads(meta["dims"])), int(meta["start_layer"]), int(meta["end_layer"]), None


def group_split(dims: ModelDims, n_layers: int, world: int, lm_head: bool):
    """[(first local layer, count)] per rank: decode bytes balanced, lm_head on the last rank."""
    from .pipeline import balanced_split
    layer = 2 * dims.params_per_layer()
    head = 2 * dims.vocab * dims.hidden if lm_head else 0.0
    return balanced_split(n_layers, world, layer, head)


def load_sub_stage(parts_path, dims, start, profile, first_layer, n_layers, first, last, device):
    """This rank's part of a stage: global layers [first_layer, first_layer + n_layers)."""
    span = SpanRuntime(dims, first_layer, n_layers, has_embed=first, has_lm_head=last, device=device,
                       **_span_kwargs())
    if profile is not None:
        span.init_synthetic(int(parts_path.split(":")[1]), profile)
        return _make_stage(span, first, last)
    from safetensors import safe_open
    with safe_open(parts_path, framework="pt", device="cpu") as f:
        for key in f.keys():
            if key.startswith("layers."):
                _, j, *rest = key.split(".")
                g = start + int(j)
                if first_layer <= g < first_layer + n_layers:
                    span.set_weight(g - first_layer, rest[-2], f.get_tensor(key))
            elif (key == "embed.weight" and first) or (key in ("norm.weight", "lm_head.weight") and last):
                span.set_weight(-1, {"embed.weight": "embed_tokens", "norm.weight": "norm",
                                     "lm_head.weight": "lm_head"}[key], f.get_tensor(key))
    return _make_stage(span, first, last)


class SpanGroup(PartitionedQwen2):
    """PartitionedQwen2's node API (same constructor arguments, same forward) over a group of
    ranks; construct it on every rank of `group` (default: the world)."""

    def __init__(self, model_name: str, num_stages: int, stage: int, parts_path: str, group=None):
        import torch.distributed as dist
        self.dist, self.group = dist, group
        self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        self.ranks = dist.get_process_group_ranks(group) if group is not None else list(range(self.world))
        self.stage, self.num_stages, self.parts_path = stage, num_stages, parts_path
        if not torch.cuda.is_available():
            raise RuntimeError("SpanGroup (inferd_amd) runs on MI355X GPUs; no CPU path")
        self.device = torch.device("cuda", torch.cuda.current_device())
        dims, start, end, profile = stage_range(parts_path, model_name, num_stages, stage)
        self.dims = dims
        last_stage = stage == num_stages - 1
        split = group_split(dims, end - start + 1, self.world, last_stage)
        f, n = split[self.rank]
        self.first_rank_layers = split
        first = stage == 0 and self.rank == 0
        last = last_stage and self.rank == self.world - 1
        self.model = load_sub_stage(parts_path, dims, start, profile, start + f, n, first, last, self.device)
        self.span = self.model.span
        if self.rank == 0 and (stage == 0 or last_stage):
            self.tokenizer = _load_tokenizer(model_name)
        self.wire_dtype = os.environ.get("INFERD_WIRE_DTYPE", _BF16)
        self.max_sessions = int(os.environ.get("INFERD_MAX_SESSIONS", 64))
        self._sessions = OrderedDict()
        self._next_ids = None
        self._staged = dist.get_backend(group) == "gloo"

    # ---------------------------------------------------------------- transport
    def _peer(self, r):
        return self.ranks[r]

    def _send(self, t, r):
        if self._staged:
            t = t.cpu()
        self.dist.send(t.contiguous(), self._peer(r), group=self.group)

    def _recv(self, shape, dtype, r):
        if self._staged:
            buf = torch.empty(shape, dtype=dtype)
            self.dist.recv(buf, self._peer(r), group=self.group)
            return buf.to(self.device)
        buf = torch.empty(shape, dtype=dtype, device=self.device)
        self.dist.recv(buf, self._peer(r), group=self.group)
        return buf

    def _bcast(self, header):
        obj = [header]
        self.dist.broadcast_object_list(obj, src=self._peer(0), group=self.group)
        return obj[0]

    # ---------------------------------------------------------------- the hooks
    def _validate(self, requests, rows, model_in):
        """Rank 0, before anything is broadcast: the checks SpanRuntime.forward would make."""
        if not requests or any(n <= 0 for _, n in requests):
            raise ValueError("forward needs at least one request with n_new_tokens >= 1")
        keys = [k for k, _ in requests if k is not None]
        if len(set(keys)) != len(keys):
            raise ValueError("a session may appear only once per forward call")
        if self.stage == 0:
            ids = torch.as_tensor(model_in).reshape(-1)
            if ids.numel() != rows:
                raise ValueError(f"{ids.numel()} ids for {rows} request tokens")
            if int(ids.min()) < 0 or int(ids.max()) >= self.dims.vocab:   # nn.Embedding's IndexError
                raise IndexError("index out of range in self (token id outside the vocabulary)")
        elif model_in.numel() != rows * self.dims.hidden:
            raise ValueError(f"hidden rows of {tuple(model_in.shape)} for {rows} request tokens")

    @torch.no_grad()
    def _run(self, requests, model_in):
        rows = sum(n for _, n in requests)
        self._validate(requests, rows, model_in)
        self._bcast({"op": "run", "requests": requests, "rows": rows})
        out, err = self._step(requests, rows, model_in)
        if err is not None:
            for key, _ in requests:          # their pages may be half-written on some ranks
                if key is not None:
                    self._release(key)
            raise RuntimeError(f"span group: {err}")
        return out

    def _release(self, key):
        self._bcast({"op": "release", "key": key})
        self.span.release(key)

    @property
    def last_next_ids(self):
        return self._next_ids

    STATUS_WORDS = 64   # status word + the failing rank's message (UTF-8, 252 bytes)

    def _status(self, code, msg=""):
        t = torch.zeros(self.STATUS_WORDS, dtype=torch.int32)
        t[0] = code
        raw = msg.encode("utf-8", "replace")[:4 * (self.STATUS_WORDS - 1)]
        raw += b"\0" * (4 * (self.STATUS_WORDS - 1) - len(raw))
        t[1:] = torch.frombuffer(bytearray(raw), dtype=torch.int32)
        return t.to(self.device)

    @staticmethod
    def _status_msg(t):
        t = t.cpu()
        return int(t[0]), bytes(t[1:].numpy().tobytes()).rstrip(b"\0").decode("utf-8", "replace")

    @torch.no_grad()
    def _step(self, requests, rows, model_in=None):
        """This rank's share of one request: input from the previous rank (rank 0: model_in),
        output to the next (the group's last rank: result back to rank 0), each hand-off a
        status word then the rows.  Never raises on a compute fault: returns (output on rank 0
        or None, error message or None)."""
        h = self.dims.hidden
        W, r = self.world, self.rank
        last_stage = self.stage == self.num_stages - 1
        code, msg = 0, ""
        if r > 0:
            code, msg = self._status_msg(self._recv((self.STATUS_WORDS,), torch.int32, r - 1))
            model_in = self._recv((rows, h), torch.bfloat16, r - 1)
        out = None
        if code == 0:
            try:
                out = self.model.run(requests, model_in)
                self.span.check_errors()
            except Exception as e:  # noqa: BLE001 -- reported to rank 0, the group stays in lockstep
                code, msg, out = r + 1, f"rank {r}: {type(e).__name__}: {e}", None
        if r < W - 1:
            self._send(self._status(code, msg), r + 1)
            self._send(out.reshape(rows, h) if code == 0 else torch.zeros(rows, h, dtype=torch.bfloat16, device=self.device), r + 1)
        elif r > 0:
            self._send(self._status(code, msg), 0)
            if last_stage:
                self._send(self.model.last_next_ids if code == 0 else torch.zeros(len(requests), dtype=torch.int32, device=self.device), 0)
            else:
                self._send(out.reshape(rows, h) if code == 0 else torch.zeros(rows, h, dtype=torch.bfloat16, device=self.device), 0)
        if r != 0:
            return None, (msg or None)
        if W > 1:
            if code == 0:     # rank 0's own failure is already known; the chain's is read back
                code, msg = self._status_msg(self._recv((self.STATUS_WORDS,), torch.int32, W - 1))
            else:
                self._recv((self.STATUS_WORDS,), torch.int32, W - 1)
            if last_stage:
                ids = self._recv((len(requests),), torch.int32, W - 1)
                if code == 0:
                    self._next_ids = ids
                return None, (msg or None) if code else None
            res = self._recv((rows, h), torch.bfloat16, W - 1)
            return (res if code == 0 else None), (msg or None) if code else None
        if last_stage and code == 0:
            self._next_ids = self.model.last_next_ids
        return out, (msg or None) if code else None

    def serve_forever(self):
        """Ranks 1..: follow rank 0's requests until shutdown()."""
        assert self.rank != 0
        while True:
            hdr = self._bcast(None)
            if hdr["op"] == "stop":
                return
            if hdr["op"] == "release":
                self.span.release(hdr["key"])
            elif hdr["op"] == "run":
                self._step(hdr["requests"], hdr["rows"])

    def shutdown(self):
        if self.rank == 0 and self.world > 1:
            self._bcast({"op": "stop"})
