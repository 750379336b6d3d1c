"""Time the leaf network's FC tail at 4096 leaves: fc1 (libazg split-K) then fc2 and
[fc3 | fc4] on hipBLASLt (round 2) or on libazg's split GEMM with a few split-K part
counts; round-robin medians of the whole forward and of the tail alone.

    python tools/fc_tail_bench.py > gpurun_out/fc_tail_bench.json
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import azg_amd  # noqa: E402,F401
from azg_amd import nnet as nn_mod  # noqa: E402


def main():
    torch.manual_seed(0)
    net = nn_mod.InflexionNNet().cuda().eval()
    B = 4096
    x = (torch.rand(B, 4, 7, 7, device="cuda") < 0.3).float()
    forms = {}
    for name, kp2, kp3 in (("hipblaslt", 0, 0), ("azg_8_4", 8, 4), ("azg_4_4", 4, 4), ("azg_8_2", 8, 2),
                           ("azg_4_2", 4, 2), ("azg_16_4", 16, 4)):
        nn_mod.FC2_KPARTS, nn_mod.FC34_KPARTS = max(kp2, 1), max(kp3, 1)
        f = nn_mod.InferenceNet(net)
        if not kp2:
            f.fc_tail_azg = False
        forms[name] = f
    ref = None
    with torch.no_grad():
        logp, _ = net(x)
        ref = torch.exp(logp)
        for f in forms.values():
            f(x)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ms = {k: [] for k in forms}
    names = list(forms)
    for r in range(7):
        order = names[r % len(names):] + names[:r % len(names)]
        for k in order:
            torch.cuda.synchronize()
            a.record()
            with torch.no_grad():
                for _ in range(5):
                    forms[k](x)
            b.record()
            b.synchronize()
            ms[k].append(a.elapsed_time(b) / 5)
    out = {}
    with torch.no_grad():
        for k, f in forms.items():
            p, _ = f(x)
            out[k] = {"forward_ms_median": sorted(ms[k])[3], "forward_ms_min": min(ms[k]),
                      "max_rel_err_P": float(((p - ref).abs() / ref).max())}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
