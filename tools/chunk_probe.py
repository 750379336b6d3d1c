"""Probe: does the 4096-leaf forward gain from running in leaf chunks whose Winograd
V / M workspaces stay inside the 256 MiB Infinity Cache?  Times InferenceNet on the whole
batch and on consecutive chunks of it (same stream, same workspace), HIP events.

    python tools/chunk_probe.py > gpurun_out/chunk_probe.json
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from azg_amd.nnet import InferenceNet, InflexionNNet  # noqa: E402


def main():
    torch.manual_seed(0)
    net = InflexionNNet().cuda().eval()
    fast = InferenceNet(net)
    B = 4096
    x = torch.randint(0, 2, (B, 4, 7, 7), device="cuda").float()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    res = {}
    with torch.no_grad():
        for chunk in (4096, 2048, 1024, 512, 256, 4096):
            def run():
                for s in range(0, B, chunk):
                    fast(x[s:s + chunk])
            for _ in range(3):
                run()
            ts = []
            for _ in range(7):
                torch.cuda.synchronize()
                ev[0].record()
                run()
                ev[1].record()
                ev[1].synchronize()
                ts.append(ev[0].elapsed_time(ev[1]))
            ts.sort()
            res[f"chunk{chunk}"] = ts[len(ts) // 2]
            print(chunk, ts[len(ts) // 2], flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
