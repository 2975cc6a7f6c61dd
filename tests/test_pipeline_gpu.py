"""The pipeline schedule with the real HIP spans on the GPU (ranks over gloo, so that it runs
on a one-GPU box: every rank shares cuda:0 and the hand-offs are staged through host memory;
the 8-GPU RCCL run is the driver's).  Covers what the CPU gloo test cannot: SpanRuntime spans
of a split model, captured decode graphs fed from exchanged buffers, the ids ring.  The
greedy ids that reach stage 0 must equal a single-stage run of the same synthetic model.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

SEED = 1234
B, T, N_STEPS = 3, 20, 5


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


# vocab-parallel head shards of the tiny model (vocab 1024) per stage count (a stage may own none)
HEAD_SHARDS = {2: [(0, 512), (512, 512)], 3: [(0, 384), (384, 0), (384, 640)]}


def _worker(rank, world, port, sizes, q, n_mb=None, sharded=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from inferd_amd.pipeline import PipelineStage
    from inferd_amd.runtime import MODELS
    d = MODELS["tiny"]
    n_mb = n_mb or world
    spans = [(sum(sizes[:i]), n) for i, n in enumerate(sizes)]
    first, n = spans[rank]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    st = PipelineStage(d, rank, world, first, n, device=dev, seed=SEED, n_microbatches=n_mb, batch=B,
                       max_ctx=T + N_STEPS + 8, prefill_chunk=2, sharded_head=sharded,
                       head_shard=HEAD_SHARDS[world][rank] if sharded else (0, 0))
    g = torch.Generator().manual_seed(7)
    prompts = [torch.randint(0, d.vocab, (B, T), generator=g) for _ in range(n_mb)]
    st.prefill(prompts)
    st.prepare_decode(N_STEPS)
    rec = []
    st.decode(2, record=rec)
    st.decode(N_STEPS - 2, record=rec)
    torch.cuda.synchronize()
    if rank == 0:
        q.put([(k, m, t.cpu().tolist()) for k, m, t in rec])
    dist.barrier()
    st.release()
    dist.destroy_process_group()


def _run(world, sizes, n_mb=None, sharded=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, sizes, q, n_mb, sharded)) for r in range(world)]
    for p in procs:
        p.start()
    rec = q.get(timeout=180)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return rec


@pytest.mark.gpu
@pytest.mark.parametrize("sizes,n_mb,sharded", [([2, 2], 2, False), ([1, 3], 3, False), ([1, 1, 2], 4, False),
                                                ([2, 2], 5, True), ([1, 1, 2], 7, True)],
                         ids=["2x2", "1-3_slack", "1-1-2_slack", "2x2_vocab_head", "1-1-2_vocab_head"])
def test_gpu_pipeline_matches_single_stage(sizes, n_mb, sharded):
    """The asynchronous ring (n_mb = S: no slack; S + 1: bench.py's default) and the vocab-parallel
    head (n_mb = 2S + 1; the last stage's final norm, shards on every stage, one owning none) with
    HIP spans: the ids fed back to stage 0 are a single span's."""
    world = len(sizes)
    got = _run(world, sizes, n_mb, sharded)
    one = _run_single_with_mb(n_mb)
    assert len(got) == N_STEPS * n_mb
    assert got == one


def _worker_single(port, n_mb, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=0, world_size=1)
    from inferd_amd.pipeline import PipelineStage
    from inferd_amd.runtime import MODELS
    d = MODELS["tiny"]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    # one stage holding every layer; n_microbatches must equal the world size (1), so the
    # microbatches of the multi-stage run are replayed one after another
    recs = []
    g = torch.Generator().manual_seed(7)
    prompts = [torch.randint(0, d.vocab, (B, T), generator=g) for _ in range(n_mb)]
    for m in range(n_mb):
        st = PipelineStage(d, 0, 1, 0, d.layers, device=dev, seed=SEED, n_microbatches=1, batch=B,
                           max_ctx=T + N_STEPS + 8, prefill_chunk=2)
        st.prefill([prompts[m]])
        st.prepare_decode(N_STEPS)
        rec = []
        st.decode(N_STEPS, record=rec)
        torch.cuda.synchronize()
        recs.append([(k, t.cpu().tolist()) for k, _, t in rec])
        st.release()
    # interleave as the ring records them: step-major, then microbatch
    q.put([(k, m, recs[m][k][1]) for k in range(N_STEPS) for m in range(n_mb)])
    dist.destroy_process_group()


def _run_single_with_mb(n_mb):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker_single, args=(_free_port(), n_mb, q))
    p.start()
    rec = q.get(timeout=180)
    p.join(timeout=120)
    assert p.exitcode == 0
    return rec
