"""Why the projection's first stage runs slower per layer than the same layers elsewhere
(bench.stage_projection: 0..4 0.532 ms vs 5..9 0.512 ms; 0..8 0.954 vs 9..17 0.912): the same
ranges timed by bench.stage_ms with and without the embedding (first=True prefills from random ids
and steps token 0; first=False prefills and steps gaussian hidden rows), interleaved.
usage: python tools/stage0_probe.py [--only LABEL:first] [--rounds 3]"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--only", default=None)
    p.add_argument("--rounds", type=int, default=3)
    a = p.parse_args()
    import bench
    from inferd_amd.pipeline import StageRange
    from inferd_amd.runtime import MODELS
    d = MODELS["qwen3-8b"]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cases = [("0..4", True), ("0..4", False), ("5..9", False), ("31..35", False)]
    if a.only:
        lab, f = a.only.split(":")
        cases = [(lab, f == "1")]
    res = {f"{lab}{' embed' if f else ''}": [] for lab, f in cases}
    for _ in range(a.rounds):
        for lab, f in cases:
            g = torch.Generator().manual_seed(11)
            ms = bench.stage_ms(d, StageRange.from_label(lab), f, False, 16, 2048, dev, g, 1234, 3, 20)
            res[f"{lab}{' embed' if f else ''}"].append(round(ms, 4))
            print(lab, f, round(ms, 4), flush=True)
    print(json.dumps({k: {"runs": v, "median": sorted(v)[len(v) // 2]} for k, v in res.items()}))


if __name__ == "__main__":
    main()
