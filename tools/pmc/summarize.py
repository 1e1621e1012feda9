"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE CSVs (separate passes) into per-kernel HBM traffic.

Corrections (MI355X_MICROARCH.md §HBM, checked with tools/pmc/calib.hip on the box):
  FETCH_SIZE counts 1/2 of the bytes of contiguous streaming reads (8 B/lane and 16 B/lane alike),
  and all bytes of 64-byte row-segment reads; WRITE_SIZE is exact.  Units are KB (1024 B).
usage: python tools/pmc/summarize.py gpurun_out/pmc profiles/<round>_pmc_summary.json
"""
import collections
import csv
import json
import os
import sys


def load(path):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        agg[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}, {k: len(v) for k, v in agg.items()}


def main(src, dst):
    f_cal, _ = load(os.path.join(src, "calib_FETCH_SIZE", "run_counter_collection.csv"))
    w_cal, _ = load(os.path.join(src, "calib_WRITE_SIZE", "run_counter_collection.csv"))
    gib_kb = float(1 << 20)
    cal = {}
    for name in f_cal:
        for tag in ("calib_copy8nt", "calib_copy8", "calib_copy16", "calib_cols"):
            if name.startswith(tag):
                cal[tag] = {"fetch_factor": gib_kb / f_cal[name], "write_factor": gib_kb / w_cal[name]}
                break
    fetch, nf = load(os.path.join(src, "bench_FETCH_SIZE", "run_counter_collection.csv"))
    write, nw = load(os.path.join(src, "bench_WRITE_SIZE", "run_counter_collection.csv"))
    # C3 bench workload: 64x3x1024x1024 fp32 pixels
    npx = 64 * 3 * 1024 * 1024
    out = {"calibration": cal, "workload": "bench.py --config c3 (64x3x1024^2, 21x21 PSF, 50 it)", "kernels": {}}
    for name in fetch:
        if "admm::" not in name:
            continue
        short = name.split("(")[0].replace("void admm::", "").replace("admm::", "")
        # row kernels stream contiguous 512-B wave segments; pass A with non-temporal loads
        ff = cal["calib_copy8"]["fetch_factor"]
        if short.startswith("k_pass_a") and "calib_copy8nt" in cal:
            ff = cal["calib_copy8nt"]["fetch_factor"]
        alg = None
        if short.startswith("k_pass_a") and short.endswith("false, false, false>"):
            alg = 28 * npx
        elif short.startswith("k_pass_a"):
            alg = 20 * npx
        elif short.startswith("k_pass_b") and short.endswith(", 0>"):
            alg = 8 * npx
        if short.startswith("k_pass_b"):
            ff = None  # 64-B column segments of sibling blocks: factor between 1 and 2 (ambiguous)
        rec = {"launches": nf[name], "fetch_KB_raw": fetch[name], "write_KB_raw": write.get(name),
               "algorithmic_bytes": alg}
        if ff is not None and write.get(name) is not None:
            t = fetch[name] * 1024 * ff + write[name] * 1024
            rec["traffic_bytes"] = t
            if alg:
                rec["traffic_over_algorithmic"] = t / alg
        else:
            lo = fetch[name] * 1024 + (write.get(name) or 0) * 1024
            rec["traffic_bytes_range"] = [lo, fetch[name] * 2048 + (write.get(name) or 0) * 1024]
        out["kernels"][short] = rec
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
