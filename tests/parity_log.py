"""Parity records of a GPU test run (errors, top-1 margins, greedy agreement), written as one
JSON file when the session ends: $INFERD_PARITY_OUT, default gpurun_out/parity.json under
the repo root (a gpurun call merges gpurun_out/ back; profiles/parity_rNN.json is the
committed copy).  Error metrics of a bf16 tensor `got` against the reference `ref`:
  max_abs   max |got - ref|
  max_norm  max_abs / max |ref|            (the tolerance the tests assert)
  rms_rel   sqrt(mean((got - ref)^2) / mean(ref^2))
  ulp_gt1   fraction of elements more than one bf16 ulp of |ref| apart
  exact     fraction of elements bit-identical"""
import json
import math
import os

import torch

RECORDS = []


def errs(got, ref) -> dict:
    g = got.detach().float().cpu().reshape(-1)
    r = ref.detach().float().cpu().reshape(-1)
    d = (g - r).abs()
    ulp = r.abs().clamp_min(1e-30) * 2.0 ** -7       # bf16 spacing at |ref| (upper bound)
    return {"max_abs": float(d.max()), "max_norm": float(d.max() / r.abs().max().clamp_min(1e-12)),
            "rms_rel": float(math.sqrt(float((d * d).mean()) / max(float((r * r).mean()), 1e-30))),
            "ulp_gt1": float((d > ulp).float().mean()), "exact": float((d == 0).float().mean()), "n": int(d.numel())}


def record(test: str, **kv):
    RECORDS.append({"test": test, **kv})


def write(root: str):
    if not RECORDS:
        return None
    path = os.environ.get("INFERD_PARITY_OUT") or os.path.join(root, "gpurun_out", "parity.json")
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as f:
        json.dump({"records": RECORDS}, f, indent=1)
    return path
