"""Lab: does a stage's measured decode time depend on what ran before it?  Measures the
sublayer8 stages in the order 0, 1, 7, 0, 3, 0, 6, 0 with bench.stage_ms (stage 0 is the
pipeline's tick in every projection)."""
import json, sys, os, time
sys.path.insert(0, "/root/repo") if os.path.exists("/root/repo") else None
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import torch
import bench
from inferd_amd.runtime import MODELS
d = MODELS["qwen3-8b"]
dev = torch.device("cuda", 0); torch.cuda.set_device(dev)
rs = bench.sub_split(d, 8, True)
g = torch.Generator(device="cpu").manual_seed(5)
res = []
for i in (0, 1, 7, 0, 3, 0, 6, 0):
    ms = bench.stage_ms(d, rs[i], i == 0, i == 7, 16, 2048, dev, g, 1234)
    res.append((rs[i].label(), round(ms * 1e3, 1)))
    print(res[-1], file=sys.stderr, flush=True)
print(json.dumps(res))
