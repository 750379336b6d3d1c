"""Probe: libazg f32-MFMA implicit-GEMM conv variants (fused bias+ReLU) vs MIOpen conv + bias + ReLU."""
import ctypes
import json
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
import azg_amd  # noqa: E402
from azg_amd import _lib  # noqa: E402


def azg_conv(x, wt, b, pad, variant):
    B, H, _, C = x.shape
    N = wt.shape[1]
    Ho = H + 2 * pad - 2
    y = torch.empty((B, Ho, Ho, N), device=x.device, dtype=torch.float32)
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    _lib.check(_lib.lib().azg_conv3x3_variant(variant, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(wt.data_ptr()),
                                              ctypes.c_void_p(b.data_ptr()), ctypes.c_void_p(y.data_ptr()),
                                              B, H, pad, C, N, s))
    return y


def t(fn, it=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s = time.perf_counter()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - s) / it


def main():
    torch.manual_seed(0)
    res = {}
    C = N = 512
    w = torch.randn(N, C, 3, 3, device="cuda") * 0.02
    b = torch.randn(N, device="cuda") * 0.1
    wt = w.permute(2, 3, 1, 0).reshape(9 * C, N).contiguous()
    variants = [int(v) for v in (sys.argv[1].split(",") if len(sys.argv) > 1 else "0,1,2,3".split(","))]
    for B in [256, 4096]:
        for H, pad in [(7, 1), (7, 0), (5, 0)]:
            x = torch.relu(torch.randn(B, H, H, C, device="cuda"))
            xn = x.permute(0, 3, 1, 2)  # channels_last view (NCHW logical)
            ref = torch.relu(F.conv2d(xn, w, b, padding=pad)).permute(0, 2, 3, 1).contiguous()
            Ho = H + 2 * pad - 2
            flops = 2 * B * Ho * Ho * N * 9 * C
            tm = t(lambda: torch.relu_(F.conv2d(xn, w, b, padding=pad)))
            row = {"miopen_tf": flops / tm / 1e12}
            for v in variants:
                got = azg_conv(x, wt, b, pad, v)
                err = ((got - ref).abs() / (ref.abs() + 1e-3)).max().item()
                ta = t(lambda: azg_conv(x, wt, b, pad, v))
                row[f"v{v}_tf"] = flops / ta / 1e12
                row[f"v{v}_err"] = err
            key = f"B{B}_H{H}_p{pad}"
            res[key] = row
            print(key, json.dumps({k: round(v, 6 if "err" in k else 1) for k, v in row.items()}), flush=True)
    json.dump(res, open("gpurun_out/conv_probe.json", "w"), indent=1)


if __name__ == "__main__":
    main()
