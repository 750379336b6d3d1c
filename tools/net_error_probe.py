"""Probe: end-to-end error of each InferenceNet conv form against the reference
module (torch.manual_seed(0) weights, the golden planes), relative to the
north_star tolerance (1e-5 on P and v)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import azg_amd  # noqa: E402,F401
import oracle_lib as ol  # noqa: E402
from azg_amd.nnet import InferenceNet, InflexionNNet  # noqa: E402


def main():
    d = dict(np.load(os.path.join(ol.GOLDEN, "nnet_golden.npz")))
    torch.manual_seed(0)
    net = InflexionNNet().eval()
    x = torch.from_numpy(d["planes"].astype(np.float32))
    P, v = d["P"].astype(np.float64), d["v"].astype(np.float64)
    # batch the 64 golden planes up to 4096 leaves (Winograd engages at >= 64)
    xb = x.repeat(64, 1, 1, 1).cuda()
    for conv in ("miopen", "azg", "winograd"):
        fast = InferenceNet(net.cuda(), conv=conv).cuda()
        with torch.no_grad():
            p, vv = fast(xb)
        p = p[:64].double().cpu().numpy()
        vv = vv[:64].double().cpu().numpy().ravel()
        ep = np.max(np.abs(p - P) / np.maximum(np.abs(P), 1e-30))
        ev = np.max(np.abs(vv - v) / np.maximum(np.abs(v), 1e-30))
        print(f"{conv:9s} max rel err P {ep:.3e}  v {ev:.3e}  (tolerance 1e-5)", flush=True)


if __name__ == "__main__":
    main()
