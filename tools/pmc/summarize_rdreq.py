"""Per-kernel HBM bytes from tools/pmc/run_rdreq.sh (request-size counters, no calibration factor):
read = 32 n32 + 64 n64 + 128 n128, write = 64 n64w + 32 (nw - n64w).  Prints per kernel: launches,
bytes per launch and, for the ADMM passes, the ratio to the algorithmic bytes (bench.py)."""
import collections
import csv
import glob
import json
import os
import sys

OUT = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/rdreq"
ALG = {  # algorithmic bytes per launch at C3 (P H W = 201,326,592 px): DESIGN.md §4
    "k_pass_a<512, false, false, false>": 28 * 201326592,
    "k_pass_a<512, false, true, false>": 20 * 201326592,
    "k_pass_b<1024, 8, 0>": 8 * 201326592,
}


def load(tag):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    launches = collections.defaultdict(set)
    for f in glob.glob(os.path.join(OUT, tag, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            short = k.split("(")[0].replace("void ", "").replace("admm::", "").replace("(anonymous namespace)::", "")
            agg[short][r["Counter_Name"]] += float(r["Counter_Value"])
            launches[short].add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
    return agg, launches


def main():
    res = {}
    for kind in ("calib", "bench"):
        rd, nl = load(kind + "1")
        wr, _ = load(kind + "2")
        for k in rd:
            n = max(len(nl[k]), 1)
            c = rd[k]
            n32, n64, n128 = (c.get("TCC_EA0_RDREQ_32B_sum", 0), c.get("TCC_EA0_RDREQ_64B_sum", 0),
                              c.get("TCC_EA0_RDREQ_128B_sum", 0))
            rbytes = (32 * n32 + 64 * n64 + 128 * n128) / n
            w = wr.get(k, {})
            nw, nw64 = w.get("TCC_EA0_WRREQ_sum", 0), w.get("TCC_EA0_WRREQ_64B_sum", 0)
            wbytes = (64 * nw64 + 32 * (nw - nw64)) / n
            e = {"launches": n, "read_bytes": rbytes, "write_bytes": wbytes,
                 "req_total_vs_sizes": (c.get("TCC_EA0_RDREQ_sum", 0) / max(n32 + n64 + n128, 1)),
                 "read_req_mix": {"32B": n32 / n, "64B": n64 / n, "128B": n128 / n}}
            if k in ALG:
                e["algorithmic_bytes"] = ALG[k]
                e["traffic_over_algorithmic"] = (rbytes + wbytes) / ALG[k]
            res[f"{kind}:{k}"] = e
    for k, e in sorted(res.items()):
        if e["read_bytes"] + e["write_bytes"] < 1e7:
            continue
        print(f"{k[:60]:60s} n={e['launches']:4d} read {e['read_bytes'] / 1e9:7.3f} GB  write {e['write_bytes'] / 1e9:7.3f} GB"
              + (f"  / alg {e['traffic_over_algorithmic']:.3f}" if "traffic_over_algorithmic" in e else "")
              + f"  mix32/64/128 {e['read_req_mix']['32B']:.3g}/{e['read_req_mix']['64B']:.3g}/{e['read_req_mix']['128B']:.3g}"
              + f"  sum-check {e['req_total_vs_sizes']:.3f}")
    with open(os.path.join(OUT, "summary.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
