"""The pipeline schedule (inferd_amd/pipeline.py) on CPU ranks over gloo.

Each rank runs its span with an oracle executor (tiny Qwen3, fp32, cached decode), so the
test checks the multi-rank schedule itself: prefill chunking, the lockstep ring exchange,
microbatch bookkeeping and the ids ring last -> first.  The greedy ids that reach stage 0
must equal a single-process oracle run of the same model.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import qwen3_ref as R

SEED = 1234


class OracleExecutor:
    """CPU stand-in for SpanExecutor: same interface, oracle compute (bf16).  sharded / head: a
    vocab-parallel head -- the last span ends with the final norm (its hand-off: the normed last
    rows, fragment-packed) and this span owns lm_head rows [head[0], head[0] + head[1])."""

    def __init__(self, d, r, first_span, last_span, sharded=False, head=(0, 0)):
        self.sp = R.RefSpan(d, SEED, r.first_layer, r.last_layer, first_span, last_span and not sharded,
                            torch.bfloat16, "sdpa",
                            skip_first_attn=r.skip_first_attn, skip_last_mlp=r.skip_last_mlp,
                            o_split_first=r.first_o, o_split_last=r.last_o, qkv_split_first=r.first_q,
                            qkv_split_last=r.last_q, final_norm_out=last_span and sharded)
        self.device = torch.device("cpu")
        self.has_embed, self.has_lm_head = first_span, last_span and not sharded
        self.dims = d
        self.r = r
        self.head_first, self.head_rows = head
        self.lm = R.gen_global_weights(d, SEED)["lm_head"][head[0]:head[0] + head[1]] if head[1] else None

    def head(self, normed, rows, keys_in=None, keys_out=None, ids=None):
        from inferd_amd.pipeline import unpack_rows
        k = R.head_keys(unpack_rows(normed.reshape(-1), rows, self.dims.hidden), self.lm, self.head_first, keys_in)
        if keys_out is not None:
            keys_out.copy_(k)
        if ids is not None:
            ids.copy_(R.keys_to_ids(k))

    @staticmethod
    def combine(keys, n_parts, rows, ids):
        ids.copy_(R.keys_to_ids(keys.reshape(n_parts, rows)))

    def _run(self, sessions, n, ids=None, x=None, want_ids=False):
        """Decode-sized hand-offs across a gate/up boundary are records (h1 first, then the packed
        SwiGLU product): the oracle reads and writes the h1 part and recomputes the whole MLP.
        Across an attention|o boundary every hand-off is a record (x, then the attention output,
        fragment-packed in a pure decode call): the oracle reads / writes both parts.  Across a
        q/k/v|attention boundary a pure decode call's hand-off is (x, raw q/k/v rows), others x."""
        from inferd_amd.pipeline import pack_rows, unpack_rows
        outs = []
        S, rows, h = len(sessions), len(sessions) * n, self.dims.hidden
        Hd = self.dims.heads * self.dims.head_dim
        packed = n == 1 and rows <= 64
        Nq = (self.dims.heads + 2 * self.dims.kv_heads) * self.dims.head_dim
        a_in = q_in = None
        if x is not None and self.r.first_o:
            tail = x.reshape(-1)[rows * h:]
            a_in = (unpack_rows(tail, rows, Hd) if packed else tail[:rows * Hd].view(rows, Hd)).reshape(S, n, Hd)
        if x is not None and self.r.first_q and n == 1:
            q_in = x.reshape(-1)[rows * h:rows * (h + Nq)].view(S, n, Nq)
        for i, sid in enumerate(sessions):
            if ids is not None:
                inp = ids.reshape(S, n)[i:i + 1].long()
                o = self.sp.forward_cached(sid, inp)
            else:
                xi = x.reshape(-1)[:rows * h].reshape(S, n, -1)[i:i + 1]
                if self.r.first_o:
                    xi = (xi, a_in[i:i + 1])
                elif self.r.first_q:
                    xi = (xi, None if q_in is None else q_in[i:i + 1])
                o = self.sp.forward_cached(sid, xi)
            outs.append(o)
        if self.sp.last:
            return torch.stack([torch.argmax(o[0, -1]) for o in outs]).to(torch.int32)
        if self.sp.final_norm_out:     # the normed last rows, fragment-packed (16-row tiles)
            p = pack_rows(torch.cat([o[0] for o in outs]).to(torch.bfloat16))
            return torch.cat([p, torch.zeros((S + 15) // 16 * 16 * h - p.numel(), dtype=torch.bfloat16)])
        if self.r.last_o:
            xs = torch.cat([o[0][0] for o in outs]).to(torch.bfloat16).reshape(-1)
            a = torch.cat([o[1][0] for o in outs]).to(torch.bfloat16)
            return torch.cat([xs, pack_rows(a) if packed else a.reshape(-1)])
        if self.r.last_q:
            xs = torch.cat([o[0][0] for o in outs]).to(torch.bfloat16)
            if n != 1:
                return xs
            return torch.cat([xs.reshape(-1), torch.cat([o[1][0] for o in outs]).to(torch.bfloat16).reshape(-1)])
        h1 = torch.cat([o[0] for o in outs]).to(torch.bfloat16)
        if self.r.last_col and rows <= 64:
            from inferd_amd.pipeline import record_elems
            rec = torch.zeros(record_elems(self.dims, rows), dtype=torch.bfloat16)
            rec[:rows * h] = h1.reshape(-1)
            return rec
        return h1

    def prefill(self, sessions, n_tokens, ids=None, x=None, want_ids=False):
        return self._run(sessions, n_tokens, ids=ids, x=x)

    def prepare_decode(self, microbatches, n_steps, bufs):
        self.mbs, self.bufs = microbatches, bufs

    def decode(self, m):
        b = self.bufs[m]
        out = self._run(self.mbs[m], 1, ids=b["ids"], x=b["x"])
        dst = b["next_ids"] if self.sp.last else b["hidden_out"]
        dst.reshape(-1)[:out.numel()].copy_(out.reshape(-1))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _split(d, world, sizes):
    """StageRanges per stage: even (bench.even_split) or the given sizes in layers (BASELINE
    config 4's uneven, balance.py-like split; multiples of 0.5 cut between a layer's attention
    and MLP halves; bench.py --spans), or "gateup": gate/up boundaries inside layers 1 and 2
    (tiny: intermediate 512, columns 256 and 128)."""
    from inferd_amd.pipeline import StageRange, even_split, ranges_from_sizes
    if sizes == "gateup":
        return [StageRange(0, 3, 0, 256), StageRange(3, 2, 256, 128), StageRange(5, 3, 128, 0)][:world]
    if sizes == "o":      # attention|o boundaries in layers 1 and 3
        return [StageRange(0, 3, last_o=True), StageRange(2, 5, first_o=True, last_o=True),
                StageRange(6, 2, first_o=True)][:world]
    if sizes == "q":          # q/k/v|attention boundaries in layers 1 and 3
        return [StageRange(0, 3, last_q=True), StageRange(2, 5, first_q=True, last_q=True),
                StageRange(6, 2, first_q=True)][:world]
    if sizes == "q_o":        # a q/k/v|attention boundary, then an attention|o one
        return [StageRange(0, 3, last_q=True), StageRange(2, 5, first_q=True, last_o=True),
                StageRange(6, 2, first_o=True)][:world]
    if sizes == "o_gateup":   # an attention|o boundary, then a gate/up one (the same stage)
        return [StageRange(0, 3, last_o=True), StageRange(2, 3, 0, 256, first_o=True), StageRange(5, 3, 256, 0)]
    if not sizes:
        return [StageRange.layers(f, n) for f, n in even_split(d.layers, world)]
    return ranges_from_sizes(sizes)


def _forced(n_mb, n_steps, vocab):
    """teacher-forcing table: ids fed at step k to microbatch m, [n_steps, n_mb, B]"""
    return torch.tensor([[[(37 * k + 11 * m + 5 * b) % vocab for b in range(3)] for m in range(n_mb)]
                         for k in range(n_steps)], dtype=torch.int32)


# vocab-parallel head shards of the tiny model (vocab 1024) per world size: (first, rows) per stage;
# a stage may own none (it passes the running keys on)
HEAD_SHARDS = {2: [(0, 384), (384, 640)], 3: [(0, 256), (256, 0), (256, 768)], 4: [(0, 0), (0, 512), (512, 256),
                                                                                  (768, 256)],
               8: [(0, 0), (0, 0), (0, 128), (128, 128), (256, 256), (512, 128), (640, 256), (896, 128)]}


def _worker(rank, world, port, n_steps, q, sizes=None, force=False, n_mb=None, sharded=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    from inferd_amd.pipeline import PipelineStage
    d = R.CONFIGS["tiny"]
    n_mb = n_mb or world
    rg = _split(d, world, sizes)[rank]
    head = HEAD_SHARDS[world][rank] if sharded else (0, 0)
    ex = OracleExecutor(d, rg, rank == 0, rank == world - 1, sharded, head)
    B = 3
    st = PipelineStage(d, rank, world, rg.first_layer, rg.n_layers, device="cpu", seed=SEED, n_microbatches=n_mb,
                       batch=B, max_ctx=64, prefill_chunk=2, executor=ex, sharded_head=sharded, head_shard=head,
                       **rg.span_kwargs())
    g = torch.Generator().manual_seed(3)
    prompts = [torch.randint(0, d.vocab, (B, 9), generator=g) for _ in range(n_mb)]
    st.prefill(prompts)
    st.prepare_decode(n_steps)
    rec = []
    if force:   # PipelineStage.decode(force=...): [steps, B] per microbatch -> this test's table
        f = _forced(n_mb, n_steps, d.vocab)
        tab = {m: f[:, m] for m in range(n_mb)}

        class ByMb:
            """force[k] for the microbatch being fed (decode() indexes force by absolute step)"""
            def __init__(self):
                self.m = 0

            def __getitem__(self, k):
                v = tab[self.m][k]
                self.m = (self.m + 1) % n_mb
                return v
        fz = ByMb()
        st.decode(2, record=rec, force=fz)
        st.decode(n_steps - 2, record=rec, force=fz)
    else:
        st.decode(2, record=rec)
        st.decode(n_steps - 2, record=rec)
    if rank == 0:
        q.put([(k, m, t.tolist()) for k, m, t in rec] + [("final", m, st.ids[m].tolist()) for m in range(n_mb)])
    dist.barrier()
    dist.destroy_process_group()


def _reference(n_mb, n_steps, sizes=None, force=False):
    """Single process: the whole model as one oracle span (no split: the stages' bf16 hand-offs,
    at layer or half-layer boundaries, are the bf16 residuals a single span computes too)."""
    d = R.CONFIGS["tiny"]
    sp = R.RefSpan(d, SEED, 0, d.layers - 1, True, True, torch.bfloat16, "sdpa")
    B = 3
    g = torch.Generator().manual_seed(3)
    prompts = [torch.randint(0, d.vocab, (B, 9), generator=g) for _ in range(n_mb)]
    feeds = {}
    f = _forced(n_mb, n_steps, d.vocab) if force else None
    for m in range(n_mb):
        for b in range(B):
            nxt = int(torch.argmax(sp.forward_cached((m, b), prompts[m][b:b + 1])[0, -1]))
            for k in range(n_steps + 1):
                if f is not None and k < n_steps:
                    nxt = int(f[k, m, b])
                feeds[(k, m, b)] = nxt
                nxt = int(torch.argmax(sp.forward_cached((m, b), torch.tensor([[nxt]]))[0, -1]))
    return feeds


def _run_ring(world, n_steps, sizes=None, force=False, n_mb=None, sharded=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_steps, q, sizes, force, n_mb, sharded))
             for r in range(world)]
    for p in procs:
        p.start()
    rec = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return rec


def _check(rec, ref, n_steps, n_mb):
    seen = 0
    for k, m, ids in rec:
        if k == "final":
            assert ids == [ref[(n_steps, m, b)] for b in range(3)]
            continue
        assert ids == [ref[(k, m, b)] for b in range(3)], (k, m)
        seen += 1
    assert seen == n_steps * n_mb


@pytest.mark.parametrize("world,sizes", [(2, None), (3, None), (3, [1, 2, 1]), (2, [3, 1]),
                                         (2, [1.5, 2.5]), (3, [0.5, 2, 1.5]), (3, "gateup"),
                                         (3, "o"), (3, "o_gateup"), (3, "q"), (3, "q_o")])
def test_pipeline_matches_single_process(world, sizes):
    """the asynchronous ring with one microbatch of slack (n_mb = S + 1, bench.py's default)"""
    n_steps, n_mb = 4, world + 1
    _check(_run_ring(world, n_steps, sizes, n_mb=n_mb), _reference(n_mb, n_steps, sizes), n_steps, n_mb)


@pytest.mark.parametrize("world,n_mb", [(2, 2), (3, 3), (3, 6)])
def test_pipeline_microbatch_counts(world, n_mb):
    """no slack (n_mb = S: the old lockstep occupancy) and a lot of it"""
    n_steps = 3
    _check(_run_ring(world, n_steps, None, n_mb=n_mb), _reference(n_mb, n_steps), n_steps, n_mb)


@pytest.mark.parametrize("world,sizes,extra", [(2, None, 1), (3, None, 1), (3, None, 0), (3, "o", 2),
                                               (4, None, 1), (3, "gateup", 1), (3, "q_o", 1)])
def test_pipeline_vocab_parallel_head(world, sizes, extra):
    """The greedy head vocab-parallel over the stages (HEAD_SHARDS: uneven, and stages owning no
    rows), the normed rows and running keys handed round the ring: the ids are the single span's
    torch.argmax over the whole vocabulary, bit for bit, at n_mb = 2S + extra microbatches."""
    n_steps, n_mb = 4, 2 * world + extra
    _check(_run_ring(world, n_steps, sizes, n_mb=n_mb, sharded=True), _reference(n_mb, n_steps, sizes), n_steps,
           n_mb)


@pytest.mark.parametrize("sharded", [False, True], ids=["whole_head", "vocab_head"])
def test_pipeline_eight_stages(sharded):
    """bench.py --gpus 8's ring on CPU ranks: the tiny model's 4 layers as eight half-layer stages
    (attention half | MLP half), S + 1 = 9 microbatches with the whole head, 2S + 1 = 17 with the
    vocab-parallel head (the first two stages owning no rows, so the running keys start on stage
    2): ids identical to one span."""
    from inferd_amd.pipeline import ring_microbatches
    world, n_steps, sizes = 8, 3, [0.5] * 8
    n_mb = ring_microbatches(world, sharded)
    assert n_mb == (17 if sharded else 9)
    _check(_run_ring(world, n_steps, sizes, n_mb=n_mb, sharded=sharded), _reference(n_mb, n_steps, sizes), n_steps,
           n_mb)


def test_pipeline_teacher_forcing():
    """PipelineStage.decode(force=...): stage 0 feeds the given ids instead of the ring's greedy
    choice at every step; the fed ids are exactly the table and the last stage's final choice is
    the single-process chain's after the same forced steps."""
    world, n_steps = 3, 4
    n_mb = world + 1
    rec = _run_ring(world, n_steps, None, True, n_mb)
    ref = _reference(n_mb, n_steps, None, force=True)
    f = _forced(n_mb, n_steps, R.CONFIGS["tiny"].vocab)
    seen = 0
    for k, m, ids in rec:
        if k == "final":
            assert ids == [ref[(n_steps, m, b)] for b in range(3)]
            continue
        assert ids == f[k, m].tolist(), (k, m)
        seen += 1
    assert seen == n_steps * n_mb
