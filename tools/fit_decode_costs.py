"""Fit the measured stage-boundary cost table (tools/boundary_costs.py) to whole-stage
measurements (bench.py --mode stages JSON files): measured stage time =
(first ? first_scale : 1) x (content_scale x content + stage + last x head_scale x head
+ first x embed), content = what the table predicts for the stage's layers and parts
(pipeline.predicted_stage_us less its stage overhead).  Writes the fit into the table's
"projection_fit" (pipeline.load_decode_costs applies it) and prints the residuals.

  python tools/fit_decode_costs.py inferd_amd/data/decode_costs_qwen3_8b.json profiles/r05/stage_projection_*.json

The table alone was measured on one box with one-layer spans; whole stages on others run
~4 % faster per layer with ~10 us more fixed cost per stage, and the first stage (embedding,
token ids) ~2.5 % slower -- what the fit absorbs.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
from scipy.optimize import least_squares  # noqa: E402

from inferd_amd import pipeline as P  # noqa: E402


def main():
    table, files = sys.argv[1], sys.argv[2:]
    with open(table) as f:
        raw = json.load(f)
    raw.pop("projection_fit", None)
    cal = P.apply_cost_fit(raw)
    rows = []
    for fn in files:
        with open(fn) as f:
            d = json.load(f)
        for name, v in d.get("stage_projection", d).items():
            if not isinstance(v, dict) or "stages" not in v:
                continue
            try:
                rs = [P.StageRange.from_label(s["range"]) for s in v["stages"]]
            except ValueError:
                continue
            for i, (r, st) in enumerate(zip(rs, v["stages"])):
                content = P.predicted_stage_us(r, cal, False, False) - cal["stage"]
                last = i == len(rs) - 1
                if "head_rows" in st:
                    # vocab-parallel head (bench.stage_projection's vhead splits): the stage's layers
                    # are its time less its shard's (head_ms); the last one ends with the final norm
                    ms = (st["ms"] - st.get("head_ms", 0.0)) * 1e3
                    rows.append((content, i == 0, False, last, ms, f"{os.path.basename(fn)}:{name}:{r.label()}"))
                else:
                    rows.append((content, i == 0, last, False, st["ms"] * 1e3,
                                 f"{os.path.basename(fn)}:{name}:{r.label()}"))
    C = np.array([r[0] for r in rows])
    F = np.array([r[1] for r in rows])
    L = np.array([r[2] for r in rows])
    N = np.array([r[3] for r in rows])
    M = np.array([r[4] for r in rows])
    norm_us = 5.5     # bench.FINAL_NORM_US: the final norm a vocab-head last stage runs

    def model(p):
        a, b, g, fs = p
        return np.where(F, fs, 1.0) * (a * C + b + L * g * cal["head"] + F * cal["embed"] + N * norm_us)
    res = least_squares(lambda p: (model(p) - M) / M, [1.0, cal["stage"], 1.0, 1.0])
    a, b, g, fs = (float(x) for x in res.x)
    fit = {"content_scale": round(a, 5), "stage": round(b, 3), "head_scale": round(g, 5), "first_scale": round(fs, 5),
           "stages": len(rows), "rms_rel": round(float(np.sqrt(np.mean(res.fun ** 2))), 5),
           "max_rel": round(float(np.abs(res.fun).max()), 5), "sources": [os.path.basename(x) for x in files]}
    raw["projection_fit"] = fit
    with open(table, "w") as f:
        json.dump(raw, f, indent=1)
    print(json.dumps(fit))
    for r, e in sorted(zip(rows, res.fun), key=lambda t: -abs(t[1]))[:12]:
        print(f"{e:+.4f} {r[5]}")


if __name__ == "__main__":
    main()
