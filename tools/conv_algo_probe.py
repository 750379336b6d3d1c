"""Probe: which MIOpen solver torch gets for the leaf network's 3x3 convolutions,
per layout (NCHW / NHWC) and find mode (torch.backends.cudnn.benchmark), with
TF/s (direct-convolution FLOPs) and the error against an f64 CPU convolution.

    python tools/conv_algo_probe.py [B] > gpurun_out/conv_algo.log
"""
import json
import sys
import time

import torch
import torch.nn.functional as F


def timeit(fn, it=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / it


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    torch.manual_seed(0)
    C = N = 512
    res = {}
    for H, pad in [(7, 1), (7, 0), (5, 0)]:
        w = torch.randn(N, C, 3, 3) * 0.02
        x = torch.relu(torch.randn(B, C, H, H))
        ref = F.conv2d(x[:32].double(), w.double(), padding=pad)
        Ho = H + 2 * pad - 2
        flops = 2 * B * Ho * Ho * N * 9 * C
        for bench in (False, True):
            torch.backends.cudnn.benchmark = bench
            for layout in ("nchw", "nhwc"):
                mf = torch.channels_last if layout == "nhwc" else torch.contiguous_format
                xg = x.cuda().contiguous(memory_format=mf)
                wg = w.cuda().contiguous(memory_format=mf)
                t = timeit(lambda: F.conv2d(xg, wg, padding=pad))
                y = F.conv2d(xg, wg, padding=pad)[:32].double().cpu()
                err = ((y - ref).abs().max() / ref.abs().max()).item()
                key = f"H{H}_p{pad}_{layout}_bench{int(bench)}"
                res[key] = {"tflops": flops / t / 1e12, "ms": t * 1e3, "max_err_rel_to_max": err}
                print(key, json.dumps(res[key]), flush=True)
    json.dump(res, open("gpurun_out/conv_algo.json", "w"), indent=1)


if __name__ == "__main__":
    main()
