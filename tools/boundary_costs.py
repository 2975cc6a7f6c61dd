"""Measure the decode-graph cost of every stage-boundary kind the splitter may cut at
(pipeline.gateup_split / sublayer_split), at Qwen3-8B, B = 16, ctx 2048, on one GPU.

Each figure is bench.stage_ms of a small span (one or five layers from the middle of the
model, synthetic weights, prefilled through the real path, its decode step replayed as a
captured graph): the splitter's cost model is built from these instead of per-kernel
means, so the cost of a boundary -- a partial gate/up GEMV writing a packed record, the
receiver's remaining columns, the first-norm launch of a stage -- is what the stage
actually pays.

  python tools/boundary_costs.py --out profiles/r05/boundary_costs.json [--step 256]

Output (us): layer (one full layer), stage (a one-layer span's time minus a layer: the
first-norm / prologue launch every stage pays), attn (span ending after layer l's attention
half), mlp[c] (span starting at layer l's MLP at gate/up column c, c = 0 the half boundary),
send[c] (span = layer l's attention half + gate/up columns [0, c)), core (attention half
without o: an attention|o boundary's sender), o_mlp (o projection + MLP: its receiver), head
(final norm + lm_head + argmax on top of one layer), embed (embedding on top of one layer),
q_send (input norm + q/k/v projection: a q/k/v|attention boundary's sender), q_recv (attention +
o + MLP: its receiver).

  --only q --merge inferd_amd/data/decode_costs_qwen3_8b.json: measure q_send / q_recv with the
  reference entries one_layer, attn, core, o_mlp beside them, and merge them into the table scaled
  by the ratio of the reference entries (the table was measured on another box).
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import bench  # noqa: E402
from inferd_amd.pipeline import StageRange  # noqa: E402
from inferd_amd.runtime import MODELS  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--model", default="qwen3-8b")
    p.add_argument("--batch", type=int, default=16)
    p.add_argument("--ctx", type=int, default=2048)
    p.add_argument("--step", type=int, default=256)
    p.add_argument("--layer", type=int, default=10)
    p.add_argument("--out", default="gpurun_out/boundary_costs.json")
    p.add_argument("--only", default="", help="q: only the q/k/v|attention boundary entries (+ references)")
    p.add_argument("--merge", default="", help="with --only: the table to merge the scaled entries into")
    a = p.parse_args()
    d = MODELS[a.model]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    g = torch.Generator(device="cpu").manual_seed(11)
    u = 2 * a.layer
    t0 = time.time()

    def ms(r, first=False, last=False):
        v = bench.stage_ms(d, r, first, last, a.batch, a.ctx, dev, g, 1234) * 1e3
        print(f"[{time.time() - t0:6.1f}s] {r.label():>16} first={int(first)} last={int(last)}: {v:8.2f} us",
              flush=True)
        return v

    if a.only == "q":
        ref = {"one_layer": ms(StageRange(u, 2)), "attn": ms(StageRange(u, 1)), "core": ms(StageRange(u, 1, last_o=True)),
               "o_mlp": ms(StageRange(u, 2, first_o=True))}
        new = {"q_send": ms(StageRange(u, 1, last_q=True)), "q_recv": ms(StageRange(u, 2, first_q=True))}
        res = {"measured": {**ref, **new}}
        if a.merge:
            with open(a.merge) as f:
                table = json.load(f)
            k = sum(table[key] for key in ref) / sum(ref.values())
            for key, v in new.items():
                table[key] = v * k
            table.setdefault("merged", []).append({"entries": sorted(new), "scale": round(k, 5), "measured": res["measured"]})
            res = table
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
        print(json.dumps(res.get("merged", res)), flush=True)
        return
    one = ms(StageRange(u, 2))
    five = ms(StageRange(u, 10))
    layer = (five - one) / 4
    res = {"model": a.model, "batch": a.batch, "ctx": a.ctx, "step": a.step, "layer": layer, "stage": one - layer,
           "one_layer": one, "five_layers": five}
    res["attn"] = ms(StageRange(u, 1))
    res["core"] = ms(StageRange(u, 1, last_o=True))
    res["o_mlp"] = ms(StageRange(u, 2, first_o=True))
    res["head"] = ms(StageRange(u, 2), last=True) - one
    res["embed"] = ms(StageRange(u, 2), first=True) - one
    res["q_send"] = ms(StageRange(u, 1, last_q=True))
    res["q_recv"] = ms(StageRange(u, 2, first_q=True))
    cols = list(range(0, d.intermediate, a.step))
    res["mlp"] = {c: ms(StageRange(u + 1, 1, c, 0)) for c in cols}
    res["send"] = {c: (ms(StageRange(u, 1, 0, c)) if c else res["attn"]) for c in cols}
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v for k, v in res.items() if not isinstance(v, dict)}), flush=True)


if __name__ == "__main__":
    main()
