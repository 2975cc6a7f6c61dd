"""Lab: does a stage's measured decode time depend on what ran before it?  Measures the
sublayer8 stages in the order 0, 1, 7, 0, 3, 0, 6, 0 with bench.stage_ms (stage 0 is the
pipeline's tick in every projection), then stages 0, 3, 7, 0 stepped eagerly (launch_eager)."""
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
order = [(0, False), (1, False), (7, False), (0, False), (3, False), (0, False), (6, False), (0, False),
         (0, True), (3, True), (7, True), (0, True)]
if len(sys.argv) > 1 and sys.argv[1] == "ab":     # graph / eager alternated on stages 3 and 0
    order = [(i, e) for _ in range(6) for i in (3, 0) for e in (False, True)]
for i, eager in order:
    ms = bench.stage_ms(d, rs[i], i == 0, i == 7, 16, 2048, dev, g, 1234, eager=eager)
    res.append((rs[i].label(), "eager" if eager else "graph", round(ms * 1e3, 1)))
    print(res[-1], file=sys.stderr, flush=True)
print(json.dumps(res))
