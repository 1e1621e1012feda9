"""Per-kernel HBM bytes from tools/pmc/run_rdreq.sh (request-size counters, no calibration factor):
read = 32 n32 + 64 n64 + 128 n128, write = 64 n64w + 32 (nw - n64w).

Writes OUT/summary.json in the format bench.py reads (profiles/<round>_pmc_summary.json): the
library's build hash (OUT/build_hash.txt, written by run_rdreq.sh from admm_tv_build_hash), the
kernels of the C3 bench with bytes per launch, the calibration copies, and the ROLES of the C3
kernels (first-iteration pass A, pass A, pass B), found from their template arguments so a rename
or a new template parameter cannot silently pair the wrong kernel with the roofline.
Usage: python tools/pmc/summarize_rdreq.py [OUT] [profiles/rNN_pmc_summary.json]"""
import collections
import csv
import glob
import json
import os
import re
import sys

OUT = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/rdreq"
DEST = sys.argv[2] if len(sys.argv) > 2 else None
# another workload (tools/pmc/run_rdreq_cfg.sh <config>): its pixels per launch, bytes per pixel reported
CFG_NPX = int(sys.argv[3]) if len(sys.argv) > 3 else None
NPX = 64 * 3 * 1024 * 1024  # C3 pixels per launch
ALG = {"pass_a_first": 20 * NPX, "pass_a": 28 * NPX, "pass_b": 8 * NPX}


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


def targs(name):
    m = re.match(r"(\w+)<(.*)>$", name.strip())
    return (m.group(1), [a.strip() for a in m.group(2).split(",")]) if m else (name, [])


def roles(kernels):
    """pass A of the aniso inference solve: k_pass_a<N, ISO=false, FIRST, HIST=false, ...>;
    pass B: the mode-0 column pass k_pass_b<H, C, 0> (or k_pass_b2) with the most launches."""
    r = {}
    for k, e in kernels.items():
        base, a = targs(k)
        if base == "k_pass_a" and len(a) >= 4 and a[1] == "false" and a[3] == "false":
            r["pass_a_first" if a[2] == "true" else "pass_a"] = k
        if base in ("k_pass_b", "k_pass_b2") and a and a[-1] == "0":
            if "pass_b" not in r or e["launches"] > kernels[r["pass_b"]]["launches"]:
                r["pass_b"] = k
    return r


def bytes_of(rd, wr, nl):
    res = {}
    for k in rd:
        n = max(len(nl[k]), 1)
        c = rd[k]
        n32, n64, n128 = (c.get("TCC_EA0_RDREQ_32B_sum", 0), c.get("TCC_EA0_RDREQ_64B_sum", 0),
                          c.get("TCC_EA0_RDREQ_128B_sum", 0))
        rbytes = (32 * n32 + 64 * n64 + 128 * n128) / n
        w = wr.get(k, {})
        nw, nw64 = w.get("TCC_EA0_WRREQ_sum", 0), w.get("TCC_EA0_WRREQ_64B_sum", 0)
        wbytes = (64 * nw64 + 32 * (nw - nw64)) / n
        res[k] = {"launches": n, "read_bytes": rbytes, "write_bytes": wbytes, "traffic_bytes": rbytes + wbytes,
                  "read_request_mix_per_launch": {"32B": n32 / n, "64B": n64 / n, "128B": n128 / n},
                  "req_total_vs_sizes": c.get("TCC_EA0_RDREQ_sum", 0) / max(n32 + n64 + n128, 1)}
    return res


def main():
    crd, cnl = load("calib1")
    calib = bytes_of(crd, load("calib2")[0], cnl)
    rd, nl = load("bench1")
    kern = bytes_of(rd, load("bench2")[0], nl)
    rl = roles(kern) if CFG_NPX is None else {}
    if CFG_NPX:
        for e in kern.values():
            e["bytes_per_pixel"] = e["traffic_bytes"] / CFG_NPX
    for role, k in rl.items():
        kern[k]["role"] = role
        kern[k]["algorithmic_bytes"] = ALG[role]
        kern[k]["traffic_over_algorithmic"] = kern[k]["traffic_bytes"] / ALG[role]
    bh = os.path.join(OUT, "build_hash.txt")
    summ = {
        "method": "rocprofv3 --pmc request-size counters, exact bytes without a calibration factor "
                  "(tools/pmc/run_rdreq.sh, tools/pmc/summarize_rdreq.py): read = 32*TCC_EA0_RDREQ_32B + "
                  "64*TCC_EA0_RDREQ_64B + 128*TCC_EA0_RDREQ_128B, write = 64*TCC_EA0_WRREQ_64B + "
                  "32*(TCC_EA0_WRREQ - TCC_EA0_WRREQ_64B), summed over TCC instances, two separate --pmc passes; "
                  "checked on calibration copies of known size. Memory-side requests include Infinity-Cache "
                  "(MALL) hits.",
        "workload": ("bench.py --config c3 (64x3x1024^2, 21x21 PSF, 50 it), 2 steps + 1 warm-up, --no-extras"
                     if CFG_NPX is None else f"tools/pmc/run_rdreq_cfg.sh ({CFG_NPX} pixels per launch), one stream"),
        "build_hash": open(bh).read().strip() if os.path.exists(bh) else None,
        "roles": rl,
        "kernels": {k: e for k, e in kern.items() if e["traffic_bytes"] > 1e4},
        "calibration": {k: e for k, e in calib.items() if e["traffic_bytes"] > 1e7},
    }
    for k, e in sorted(summ["kernels"].items(), key=lambda t: -t[1]["traffic_bytes"]):
        print(f"{k[:60]:60s} n={e['launches']:4d} read {e['read_bytes'] / 1e9:7.3f} GB  "
              f"write {e['write_bytes'] / 1e9:7.3f} GB"
              + (f"  {e['role']}: {e['traffic_over_algorithmic']:.3f} x alg" if "role" in e else "")
              + (f"  {e['bytes_per_pixel']:.2f} B/px" if "bytes_per_pixel" in e else ""))
    for k, e in summ["calibration"].items():
        print(f"calib {k[:54]:54s} read {e['read_bytes'] / 1e9:7.3f} GB  write {e['write_bytes'] / 1e9:7.3f} GB")
    with open(os.path.join(OUT, "summary.json"), "w") as f:
        json.dump(summ, f, indent=1)
    if DEST:
        with open(DEST, "w") as f:
            json.dump(summ, f, indent=1)


if __name__ == "__main__":
    main()
