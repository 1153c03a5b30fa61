#!/usr/bin/env python3
"""Per-kernel SQ-counter summary of tools/pmc_sq.sh passes (rocprofv3 --pmc CSVs).

Derived, per kernel (averaged over its dispatches):
  mfma_busy  = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs * 1024 SIMDs)  (fraction of SIMD-cycles the
               matrix pipe is busy over the dispatch; counts cycles, MI355X_MICROARCH.md constants table)
  wait_any / wait_inst / active = SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES (quad-cycle
               units all, so the ratios are unit-free; the three are disjoint and sum to about 1)
  lds_conflict = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE;  coexec = SQ_VALU_MFMA_COEXEC_CYCLES / MFMA busy cycles
  clock_ghz  = GRBM_GUI_ACTIVE / 8 / dispatch duration (reads high on dispatches < 0.3 ms, guide §DVFS)
Usage: python tools/sq_summary.py <dir_A> <dir_B> [out.json]"""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import short_name  # noqa: E402


def load(d):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per = collections.defaultdict(lambda: collections.defaultdict(float))   # (kernel, dispatch) -> counter -> sum
    dur = {}
    for r in csv.DictReader(open(f[0])):
        key = (r["Kernel_Name"], r["Dispatch_Id"])
        per[key][r["Counter_Name"]] += float(r["Counter_Value"])
        if "Start_Timestamp" in r and r.get("End_Timestamp"):
            dur[key] = (float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) * 1e-9
    return per, dur


def main():
    pa, da = load(sys.argv[1])
    pb, _ = load(sys.argv[2])
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for per in (pa, pb):
        for (k, _d), cs in per.items():
            for c, v in cs.items():
                agg[short_name(k)][c].append(v)
    durs = collections.defaultdict(list)
    for (k, _d), t in da.items():
        durs[short_name(k)].append(t)
    out = {}
    for k, cs in agg.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        n = len(cs.get("SQ_WAVE_CYCLES", [1]))
        g = m.get("GRBM_GUI_ACTIVE", 0.0)
        wc = m.get("SQ_WAVE_CYCLES", 0.0)
        r = {"dispatches": n}
        if g:
            r["mfma_busy"] = round(m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (g / 8 * 1024), 4)
        if wc:
            for name, c in (("wait_any", "SQ_WAIT_ANY"), ("wait_inst", "SQ_WAIT_INST_ANY"),
                            ("wait_inst_lds", "SQ_WAIT_INST_LDS"), ("active", "SQ_ACTIVE_INST_ANY")):
                if c in m:
                    r[name] = round(m[c] / wc, 4)
        if m.get("SQ_LDS_IDX_ACTIVE"):
            r["lds_conflict"] = round(m.get("SQ_LDS_BANK_CONFLICT", 0.0) / m["SQ_LDS_IDX_ACTIVE"], 4)
        if m.get("SQ_VALU_MFMA_BUSY_CYCLES"):
            r["coexec_per_mfma_busy"] = round(m.get("SQ_VALU_MFMA_COEXEC_CYCLES", 0.0) / m["SQ_VALU_MFMA_BUSY_CYCLES"], 4)
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_INSTS_VMEM", "SQ_INSTS_SALU"):
            if c in m:
                r[c] = m[c]
        if durs.get(k) and g:
            t = sum(durs[k]) / len(durs[k])
            r["duration_us_profiled"] = round(t * 1e6, 2)
            r["clock_ghz"] = round(g / 8 / t / 1e9, 3)
        out[k] = r
    order = sorted(out, key=lambda k: -out[k].get("duration_us_profiled", 0) * out[k]["dispatches"])
    res = {k: out[k] for k in order}
    txt = json.dumps(res, indent=1)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(txt)
    for k in order[:14]:
        r = out[k]
        print(f"{k[:70]:70s} n={r['dispatches']:4d} mfma={r.get('mfma_busy', 0):.3f} wait={r.get('wait_any', 0):.3f} "
              f"inst={r.get('wait_inst', 0):.3f} act={r.get('active', 0):.3f} ldsc={r.get('lds_conflict', 0):.3f} "
              f"clk={r.get('clock_ghz', 0):.2f} t={r.get('duration_us_profiled', 0):.1f}us")


if __name__ == "__main__":
    main()
