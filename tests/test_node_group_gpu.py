"""One petals node served by a group of GPUs (inferd_amd/node_group.py): the node API on rank
0, the stage's layers split over the group's ranks (gloo ranks sharing this box's GPU, hidden
rows staged through host memory; RCCL between GPUs of one host).  A two-stage Qwen3-0.6B chain
(peaked synthetic profile) where one stage is a group must give the same greedy ids as the
chain of two single-GPU PartitionedQwen2 nodes, stateless and with a session."""
import os
import socket

import pytest
import torch

SEED = 1234
SPECS = [f"synthetic:{SEED}:qwen3-0.6b:0:13:peaked", f"synthetic:{SEED}:qwen3-0.6b:14:27:peaked"]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _chain(n0, n1, prompt, steps, sid=None):
    ids, out = list(prompt), []
    for _ in range(steps):
        inp = {"generated_ids": ids}
        if sid is not None:
            inp["session_id"] = sid
        o1 = n1.forward(n0.forward(inp))
        out.append(o1["next_token_id"])
        ids = o1["generated_ids"]
    return out


FAIL_ROWS = 7   # a request of this many rows raises on the group's last rank (fault injection)


def _worker(rank, world, port, grouped_stage, out_path):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from inferd_amd.node_group import SpanGroup
    from inferd_amd.partitioned_models import PartitionedQwen2
    grp = SpanGroup("qwen3-0.6b", 2, grouped_stage, SPECS[grouped_stage])
    if rank != 0:
        if rank == world - 1:
            run = grp.model.run

            def faulty(requests, model_in, **kw):
                if sum(n for _, n in requests) == FAIL_ROWS:
                    raise RuntimeError("injected fault")
                return run(requests, model_in, **kw)
            grp.model.run = faulty
        grp.serve_forever()
        dist.destroy_process_group()
        return
    other = 1 - grouped_stage
    single = PartitionedQwen2("qwen3-0.6b", 2, other, SPECS[other])
    n0, n1 = (grp, single) if grouped_stage == 0 else (single, grp)
    prompt = torch.randint(0, 151936, (32,), generator=torch.Generator().manual_seed(5)).tolist()
    res = {"split": grp.first_rank_layers}
    # faults: a bad token id is refused on rank 0 before anything is broadcast; a compute fault
    # on the group's last rank comes back as rank 0's RuntimeError; the group keeps serving
    faults = []
    bad = {"generated_ids": [1, 2, 151936]} if grouped_stage == 0 else None
    if bad is not None:
        try:
            n1.forward(n0.forward(bad))
        except IndexError:
            faults.append("index")
    try:
        n1.forward(n0.forward({"generated_ids": prompt[:FAIL_ROWS]}))
    except RuntimeError as e:
        faults.append("injected" if "injected fault" in str(e) else str(e))
    res["faults"] = faults
    res["stateless"] = _chain(n0, n1, prompt, 8)
    res["session"] = _chain(n0, n1, prompt, 8, sid="g")
    n1.forward(n0.forward({"session_id": "g", "close_session": True}))
    res["free_after_close"] = grp.span.kv.n_free == grp.span.kv.n_pages
    grp.shutdown()
    ref0 = PartitionedQwen2("qwen3-0.6b", 2, 0, SPECS[0])
    ref1 = PartitionedQwen2("qwen3-0.6b", 2, 1, SPECS[1])
    res["reference"] = _chain(ref0, ref1, prompt, 8)
    torch.save(res, out_path)
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.timeout(600)
@pytest.mark.parametrize("world,grouped_stage", [(2, 0), (3, 0), (3, 1)])
def test_span_group_node_matches_single_gpu_chain(tmp_path, world, grouped_stage):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    port = _free_port()
    out = str(tmp_path / "res.pt")
    procs = [ctx.Process(target=_worker, args=(r, world, port, grouped_stage, out)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=500)
    for p in procs:
        assert p.exitcode == 0
    res = torch.load(out, weights_only=True)
    print(f"world {world}, stage {grouped_stage} grouped, split {res['split']}: {res['stateless']}")
    assert len(res["split"]) == world
    assert res["faults"] == (["index", "injected"] if grouped_stage == 0 else ["injected"]), res["faults"]
    assert res["stateless"] == res["reference"]
    assert res["session"] == res["reference"]
    assert res["free_after_close"]
