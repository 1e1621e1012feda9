"""Per-kernel SQ counters from tools/pmc/run_sq_cfg.sh (two rocprofv3 --pmc passes) -> JSON.

Per kernel: dispatches, counters per dispatch and the derived issue figures the generic-path
analysis uses: VALU / LDS / SALU / VMEM instructions per wave, the share of wave
cycles with a VALU or LDS instruction issued, LDS bank-conflict cycles per LDS instruction.
usage: python tools/pmc/summarize_sq.py gpurun_out/sq_bsd profiles/r03_sq_bsd.json
"""
import collections
import csv
import glob
import json
import os
import re
import sys


def load(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("admm::", "")
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
    return agg, disp


def main(src, dst):
    out = {}
    for p in sorted(glob.glob(os.path.join(src, "p*"))):
        if not os.path.isdir(p):
            continue
        agg, disp = load(p)
        for k, c in agg.items():
            e = out.setdefault(k, {"dispatches": len(disp[k]), "per_dispatch": {}})
            n = max(len(disp[k]), 1)
            for name, v in c.items():
                e["per_dispatch"][name] = v / n
    for k, e in out.items():
        c = e["per_dispatch"]
        waves = c.get("SQ_WAVES", 0)
        if waves:
            d = {f"{x.lower()}_per_wave": c[f"SQ_INSTS_{x}"] / waves for x in ("VALU", "LDS", "SALU", "VMEM")
                 if f"SQ_INSTS_{x}" in c}
            if c.get("SQ_WAVE_CYCLES"):
                for x in ("VALU", "LDS", "ANY"):
                    if f"SQ_ACTIVE_INST_{x}" in c:
                        d[f"active_{x.lower()}_share"] = c[f"SQ_ACTIVE_INST_{x}"] / c["SQ_WAVE_CYCLES"]
                if "SQ_WAIT_INST_LDS" in c:
                    d["wait_lds_share"] = c["SQ_WAIT_INST_LDS"] / c["SQ_WAVE_CYCLES"]
            if c.get("SQ_INSTS_LDS"):
                d["lds_bank_conflict_cycles_per_lds_inst"] = c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_INSTS_LDS"]
            e["derived"] = d
    rows = sorted(out.items(), key=lambda kv: -kv[1]["per_dispatch"].get("SQ_WAVE_CYCLES", 0))
    for k, e in rows[:12]:
        print(f"{k[:70]:70s} n={e['dispatches']:4d} " + " ".join(f"{a}={b:.3g}" for a, b in e.get("derived", {}).items()))
    with open(dst, "w") as f:
        json.dump({"source": "tools/pmc/run_sq_cfg.sh (rocprofv3 --pmc, two passes), tools/pmc/summarize_sq.py",
                   "kernels": dict(rows)}, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
