"""Probe: the FC tail at small leaf batches (C2: 256) on libazg's split GEMM with many
split-K parts (more tiles for a short launch) against the default f32 tail on hipBLASLt;
whole-forward round-robin medians and P's error against the module.

    python tools/fc_small_probe.py --batch 256 > gpurun_out/fc_small_probe.json
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import azg_amd  # noqa: E402,F401
from azg_amd import nnet as nn_mod  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--combos", default="4-4-2,9-4-2,18-8-4,36-16-8,72-16-8,36-8-4,18-16-8")
    a = ap.parse_args()
    torch.manual_seed(0)
    net = nn_mod.InflexionNNet().cuda().eval()
    B = a.batch
    x = (torch.rand(B, 4, 7, 7, device="cuda") < 0.3).float()
    x[:, 2] = 5.0
    forms = {"f32_tail": nn_mod.InferenceNet(net)}
    for c in a.combos.split(","):
        k1, k2, k3 = (int(v) for v in c.split("-"))
        nn_mod.FC1_KPARTS, nn_mod.FC2_KPARTS, nn_mod.FC34_KPARTS = k1, k2, k3
        forms[f"azg_{c}"] = nn_mod.InferenceNet(net)
    nn_mod.FC1_KPARTS, nn_mod.FC2_KPARTS, nn_mod.FC34_KPARTS = 4, 4, 2
    min_batch = nn_mod.FC1_SPLIT_MIN_BATCH

    def run(k, f):
        nn_mod.FC1_SPLIT_MIN_BATCH = min_batch if k == "f32_tail" else 0
        return f(x)

    with torch.no_grad():
        logp, _ = net(x)
        ref = torch.exp(logp)
        for k, f in forms.items():
            run(k, f)
    a_, b_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ms = {k: [] for k in forms}
    names = list(forms)
    for r in range(9):
        order = names[r % len(names):] + names[:r % len(names)]
        for k in order:
            torch.cuda.synchronize()
            a_.record()
            with torch.no_grad():
                for _ in range(20):
                    run(k, forms[k])
            b_.record()
            b_.synchronize()
            ms[k].append(a_.elapsed_time(b_) / 20)
    out = {"batch": B}
    with torch.no_grad():
        for k, f in forms.items():
            p, _ = run(k, f)
            f.check_range()
            out[k] = {"forward_us_median": sorted(ms[k])[4] * 1e3, "forward_us_min": min(ms[k]) * 1e3,
                      "max_rel_err_P": float(((p - ref).abs() / ref).max())}
    nn_mod.FC1_SPLIT_MIN_BATCH = min_batch
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
