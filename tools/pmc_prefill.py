"""Per-launch HBM traffic of the prefill kernels (BASELINE config 5: one Qwen3-32B 8-layer
stage, 8k tokens) from two rocprofv3 PMC passes, with the same gfx950 corrections as
tools/pmc_traffic.py (fetched bytes = 2 * FETCH_SIZE * 1024, also for `buffer_load ... lds`;
written bytes = WRITE_SIZE * 1024; MI355X_MICROARCH.md §HBM).  Alongside each class: the
algorithmic bytes of one launch (operands read once, output written once), so the ratio
shows how much of the L2/MALL tile re-reading reaches HBM.

  tools/pmc_prefill.sh [B]   (on the GPU box) -> profiles/traffic_prefill_rNN.json (B = 1) or
                             traffic_prefill_b<B>_rNN.json (B sequences of 8k tokens per call)
"""
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import per_dispatch  # noqa: E402

# Qwen3-32B, T = 8192 prompt tokens per sequence, B sequences per call (PMC_BATCH)
h, I, H, KV, hd, T = 5120, 25600, 64, 8, 128, 8192
B = int(os.environ.get("PMC_BATCH", "1"))


def classify(name, state):
    if "gemm_w4p_kernel" in name or "gemm_w4_kernel" in name:
        epi = int(re.search(r"gemm_w4p?_kernel<(\d+)", name).group(1))
        if epi == 5:
            return "qkv_gemm"
        if epi == 2:
            return "gateup_gemm"
        if epi == 1:
            state["resid"] ^= 1
            return "o_gemm" if state["resid"] == 1 else "down_gemm"
    if "attn_prefill_kernel" in name:
        return "attention"
    return None


def alg_bytes():
    """operands read once and outputs written once per launch (weights once per call; M = B*T rows)"""
    qkvN = (H + 2 * KV) * hd
    M = B * T
    return {
        "qkv_gemm": M * h * 2 + qkvN * h * 2 + M * H * hd * 2 + 2 * M * KV * hd * 2,
        "attention": M * H * hd * 2 + 2 * M * KV * hd * 2 + M * H * hd * 2,
        "o_gemm": M * H * hd * 2 + h * H * hd * 2 + 2 * M * h * 2,
        "gateup_gemm": M * h * 2 + 2 * I * h * 2 + M * I * 2,
        "down_gemm": M * I * 2 + h * I * 2 + 2 * M * h * 2,
    }


def summarize(seq, scale):
    acc, state = {}, {"resid": 0}
    for name, v in seq:
        c = classify(name, state)
        if c is not None:
            acc.setdefault(c, []).append(v * scale)
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    fetch = summarize(per_dispatch(sys.argv[1], "FETCH_SIZE"), 2 * 1024.0)
    write = summarize(per_dispatch(sys.argv[2], "WRITE_SIZE"), 1024.0)
    alg = alg_bytes()
    per = {k: int(fetch.get(k, 0) + write.get(k, 0)) for k in sorted(set(fetch) | set(write))}
    print(json.dumps({
        "workload": "qwen3-32b-prefill-8layers-T8192" + (f"-B{B}" if B > 1 else ""),
        "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes); bytes = 2*FETCH_SIZE*1024 "
                  "+ WRITE_SIZE*1024; mean over launches",
        "per_launch_bytes": per,
        "alg_bytes_per_launch": alg,
        "traffic_over_alg": {k: round(per[k] / alg[k], 3) for k in per if k in alg},
        "fetch_bytes": {k: int(v) for k, v in fetch.items()},
        "write_bytes": {k: int(v) for k, v in write.items()},
    }, indent=1))


if __name__ == "__main__":
    main()
