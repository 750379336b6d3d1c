"""Relative error against f64 of the trainer's FC GEMMs (forward, and the two backward products) with
the packaged TunableOp solutions (nnet.TUNABLEOP_RESULTS) and with TunableOp off.

    python tools/tunable_precision.py
"""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import azg_amd  # noqa: E402,F401
from azg_amd import nnet  # noqa: E402


def errs(b, k, n, g):
    x = torch.randn((b, k), generator=g).cuda()
    w = torch.randn((n, k), generator=g).cuda() / k ** 0.5
    bias = torch.randn((n,), generator=g).cuda()
    dy = torch.randn((b, n), generator=g).cuda()
    out = {}
    for name, f32, f64 in (("fwd", lambda: F.linear(x, w, bias), lambda: F.linear(x.double(), w.double(), bias.double())),
                           ("dx", lambda: dy @ w, lambda: dy.double() @ w.double()),
                           ("dw", lambda: dy.t() @ x, lambda: dy.double().t() @ x.double())):
        r = f64()
        out[name] = float(((f32().double() - r).norm() / r.norm()).item())
    return out


def main():
    tun = torch.cuda.tunable
    shapes = [(b, 4608, 1024) for b in (512, 256, 128, 64)] + [(b, 1024, 512) for b in (512, 256, 128, 64)] + \
             [(b, 512, 343) for b in (512, 256)]
    res = {}
    for mode in ("off", "file"):
        tun.enable(mode == "file")
        if mode == "file":
            tun.tuning_enable(False)
            res["read"] = bool(tun.read_file(nnet.TUNABLEOP_RESULTS))
        g = torch.Generator().manual_seed(0)
        res[mode] = {f"{b}x{k}x{n}": errs(b, k, n, g) for b, k, n in shapes}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
