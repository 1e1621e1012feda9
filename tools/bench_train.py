"""The default bench line's `train` key alone (bench.train_extra: one ADMMDeconv module at the C5 shape,
forward with history + backward, reverse row pass GB/s): python tools/bench_train.py [steps]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "torch-admm-deconv_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    res = bench.train_extra(torch.device("cuda", 0), steps=steps)
    from admmtor import _native
    res["build_hash"] = _native.load().admm_tv_build_hash().decode()
    print(json.dumps(res), flush=True)
