"""The one-leaf forward of the 7x7 Inflexion network (the drop-in's batch, C1) in its small-batch
forms, each timed as 20 forwards captured in one HIP graph and replayed (device time per forward,
no host launch cost): the per-layer kernels (azg_small.hip, one launch per layer) and the fused
one-launch forward (azg_small_net) at several grid sizes.  Prints one JSON line per form.

    python tools/small_net_probe.py [B]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import azg_amd  # noqa: E402,F401
from azg_amd import _lib  # noqa: E402
from azg_amd.nnet import InferenceNet, InflexionNNet  # noqa: E402
import small_probes as sp  # noqa: E402  (tools/, the script's own directory)


def graph_time(fn, x, n=20, reps=10):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn(x)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn(x)
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(reps):
        a.record()
        g.replay()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / n)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    torch.manual_seed(0)
    net = InflexionNNet(n=7, depth=4, action_size=343).cuda().eval()
    layers = InferenceNet(net, conv="miopen", gemm="f32").cuda()
    fused_ev = sp.ProbeInferenceNet(net, conv="miopen", gemm="f32", mode="fused").cuda()
    x = (torch.rand(B, 4, 7, 7, device="cuda") < 0.3).float()
    L = sp.lib()
    with torch.no_grad():
        for form, fused, blocks in [("layers", False, 0), ("fused", True, 0), ("fused", True, 128),
                                    ("fused", True, 64), ("layers", False, 0), ("fused", True, 0)]:
            sp.check(L.azg_small_net_blocks(blocks), "azg_small_net_blocks")
            t = graph_time(fused_ev if fused else layers, x)
            print(json.dumps({"form": form, "blocks": blocks, "B": B, "us_per_forward": t}), flush=True)
        sp.check(L.azg_small_net_blocks(0), "azg_small_net_blocks")
        fused_ev.check_fused()


if __name__ == "__main__":
    main()
