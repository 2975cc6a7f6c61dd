"""Lab: the whole Qwen3-8B model as one span (36 layers + head, B = 16, ctx 2048: the bench's N = 1
workload) stepped by graph replay vs eagerly (DecodeGraph.launch vs launch_eager), alternated,
bench.stage_ms (HIP events around 20 steps after 3 warm-ups)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import bench  # noqa: E402
from inferd_amd.pipeline import StageRange  # noqa: E402
from inferd_amd.runtime import MODELS  # noqa: E402


def main():
    d = MODELS["qwen3-8b"]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    g = torch.Generator(device="cpu").manual_seed(5)
    r = StageRange(0, 2 * d.layers)
    res = []
    for eager in (False, True, False, True, False, True):
        ms = bench.stage_ms(d, r, True, True, 16, 2048, dev, g, 1234, eager=eager)
        res.append(("eager" if eager else "graph", round(ms * 1e3, 1)))
        print(res[-1], file=sys.stderr, flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
