"""MFMA utilisation of the prefill kernels (BASELINE config 5: one Qwen3-32B 8-layer stage, 8k
tokens) from one rocprofv3 SQ/GRBM counter pass plus an un-counted kernel-trace pass.

  tools/pmc_prefill_mfma.sh   (on the GPU box) -> profiles/mfma_prefill_rNN.json

Per kernel class, mean over launches:
  * mfma_busy_cycles  SQ_VALU_MFMA_BUSY_CYCLES (summed by rocprofv3 over the chip)
  * n_mfma            the launch's v_mfma_f32_16x16x32_bf16 count, from its algorithmic flops
                      (16 x 16 x 32 x 2 flops each; GEMMs are all 16x16x32 MFMAs)
  * busy_per_mfma     mfma_busy_cycles / n_mfma: the counter's cycles per MFMA
  * mfma_busy_frac    mfma_busy_cycles / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs): the share of SIMD
                      cycles the matrix pipe was busy (GRBM_GUI_ACTIVE is the sum over the 8 XCDs,
                      MI355X_MICROARCH.md, DVFS give-back)
  * clock_ghz         GRBM_GUI_ACTIVE / 8 / the traced kernel duration
  * tflops, frac_of_2500, frac_of_clock_peak   achieved rate, against the 2.5 PF/s dense bf16
                      spec and against the peak at the clock the chip held (1024 flops / cycle /
                      SIMD x 1024 SIMDs x clock)
  * valu_per_wave_cycle SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES, lds_wait_frac SQ_WAIT_INST_LDS /
                      SQ_WAVE_CYCLES (both in quad-cycles)
  * wave_cycle_split  (second pass, optional third argument) the wave cycles split into parked
                      (SQ_WAIT_ANY: s_waitcnt / barrier), issue-stalled (SQ_WAIT_INST_ANY: MFMA
                      dependency / pipe busy) and issuing (SQ_ACTIVE_INST_ANY) -- disjoint, summing
                      to SQ_WAVE_CYCLES (MI355X_MICROARCH.md, SQ counters); coexec_frac
                      SQ_VALU_MFMA_COEXEC_CYCLES / SQ_VALU_MFMA_BUSY_CYCLES (the share of matrix-busy
                      cycles with vector instructions executing beside them); lds_conflict_frac
                      SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
"""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_prefill import B, H, KV, I, T, classify, h, hd  # noqa: E402
from pmc_traffic import rows  # noqa: E402

COUNTERS = ("SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAVE_CYCLES", "SQ_ACTIVE_INST_VALU",
            "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS", "GRBM_GUI_ACTIVE")


def flops():
    qkvN = (H + 2 * KV) * hd
    M = B * T
    return {
        "qkv_gemm": 2.0 * M * qkvN * h,
        "attention": B * 4.0 * H * hd * T * (T + 1) / 2,  # causal: QK^T and PV over the lower triangle
        "o_gemm": 2.0 * M * h * H * hd,
        "gateup_gemm": 2.0 * M * 2 * I * h,
        "down_gemm": 2.0 * M * h * I,
    }


def counters(d):
    per = {}
    for r in rows(d):
        did = int(r.get("Dispatch_Id", r.get("Correlation_Id", 0)))
        e = per.setdefault(did, {"name": r.get("Kernel_Name", "")})
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return [per[k] for k in sorted(per)]


def durations(d):
    files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no kernel_trace.csv under {d}")
    out = []
    for fn in files:
        with open(fn) as f:
            for r in csv.DictReader(f):
                out.append((int(r["Start_Timestamp"]), r["Kernel_Name"],
                            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9))
    return [(n, t) for _, n, t in sorted(out)]


def by_class(seq, key):
    acc, state = {}, {"resid": 0}
    for item in seq:
        c = classify(key(item)[0], state)
        if c is not None:
            acc.setdefault(c, []).append(key(item)[1])
    return acc


def main():
    pmc = by_class(counters(sys.argv[1]), lambda e: (e["name"], e))
    pmc2 = by_class(counters(sys.argv[3]), lambda e: (e["name"], e)) if len(sys.argv) > 3 else {}
    dur = {k: sum(v) / len(v) for k, v in by_class(durations(sys.argv[2]), lambda e: e).items()}
    fl = flops()
    out = {}
    for c, launches in sorted(pmc.items()):
        m = {k: sum(e.get(k, 0.0) for e in launches) / len(launches) for k in COUNTERS}
        n_mfma = fl[c] / (16 * 16 * 32 * 2)
        cyc = m["GRBM_GUI_ACTIVE"] / 8
        t = dur.get(c)
        row = {
            "launches": len(launches),
            "counters_mean": {k: round(v) for k, v in m.items()},
            "n_mfma": round(n_mfma),
            "busy_per_mfma": round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / n_mfma, 3),
            "mfma_busy_frac": round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * 1024), 4) if cyc else None,
            "valu_per_wave_cycle": round(m["SQ_ACTIVE_INST_VALU"] / m["SQ_WAVE_CYCLES"], 4)
            if m["SQ_WAVE_CYCLES"] else None,
            "lds_wait_frac": round(m["SQ_WAIT_INST_LDS"] / m["SQ_WAVE_CYCLES"], 4) if m["SQ_WAVE_CYCLES"] else None,
        }
        if t:
            clk = cyc / t
            row.update({
                "duration_ms": round(t * 1e3, 4),
                "clock_ghz": round(clk * 1e-9, 3),
                "tflops": round(fl[c] / t * 1e-12, 1),
                "frac_of_2500": round(fl[c] / t / 2.5e15, 4),
                "frac_of_clock_peak": round(fl[c] / t / (1024 * 1024 * clk), 4),
            })
        if c in pmc2:
            l2 = pmc2[c]
            m2 = {k: sum(e.get(k, 0.0) for e in l2) / len(l2) for k in
                  ("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                   "SQ_VALU_MFMA_COEXEC_CYCLES", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE")}
            wc = m2["SQ_WAVE_CYCLES"] or 1.0
            row["counters_pass2_mean"] = {k: round(v) for k, v in m2.items()}
            row["wave_cycle_split"] = {"parked": round(m2["SQ_WAIT_ANY"] / wc, 4),
                                       "issue_stalled": round(m2["SQ_WAIT_INST_ANY"] / wc, 4),
                                       "issuing": round(m2["SQ_ACTIVE_INST_ANY"] / wc, 4)}
            row["coexec_frac"] = round(m2["SQ_VALU_MFMA_COEXEC_CYCLES"] / max(m["SQ_VALU_MFMA_BUSY_CYCLES"], 1.0), 4)
            row["lds_conflict_frac"] = round(m2["SQ_LDS_BANK_CONFLICT"] / max(m2["SQ_LDS_IDX_ACTIVE"], 1.0), 4)
        out[c] = row
    print(json.dumps({
        "workload": "qwen3-32b-prefill-8layers-T8192" + (f"-B{B}" if B > 1 else ""),
        "method": "rocprofv3 --pmc " + " ".join(COUNTERS) + " (one pass); durations from a separate "
                  "--kernel-trace pass; means over launches; see tools/pmc_prefill_mfma.py for each field",
        "classes": out,
    }, indent=1))


if __name__ == "__main__":
    main()
