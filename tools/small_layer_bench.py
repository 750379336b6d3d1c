"""Per-layer time of azg_small_conv3x3 / azg_small_fc at one leaf (C1's batch) on the 7x7 Inflexion network's
shapes, against torch's conv2d / linear (MIOpen / hipBLASLt, + bias + ReLU) on the same
inputs; medians of round-robin rounds.  Prints one JSON line per layer."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import azg_amd  # noqa: E402,F401
from azg_amd import _lib  # noqa: E402

B = int(os.environ.get("AZG_SL_B", "1"))
LAYERS = [("conv1", 7, 1, 4, 512, "nchw"), ("conv2", 7, 1, 512, 512, "nhwc"), ("conv3", 7, 0, 512, 512, "nhwc"),
          ("conv4", 5, 0, 512, 512, "nhwc"), ("fc1", 1, 0, 4608, 1024, "row"), ("fc2", 1, 0, 1024, 512, "row"),
          ("fc34", 1, 0, 512, 344, "row")]


def timeit(fn, reps=50):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    L = _lib.lib()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for name, H, pad, cin, cout, layout in LAYERS:
        taps = 9 if H > 1 else 1
        x = torch.randn(B, cin, H, H, device="cuda")
        w = torch.randn(cout, cin, 3, 3, device="cuda") if taps == 9 else torch.randn(cout, cin, device="cuda")
        b = torch.randn(cout, device="cuda")
        wk = w.contiguous(memory_format=torch.channels_last) if taps == 9 else w.contiguous()
        if layout == "nchw":
            xin, strides = x.contiguous(), (cin * H * H, H, 1, H * H)
        else:
            xin = x.permute(0, 2, 3, 1).contiguous()
            strides = (H * H * cin, H * cin, cin, 1)
        Ho = H + 2 * pad - 2 if taps == 9 else 1
        y = torch.empty((B * Ho * Ho, cout), device="cuda")

        def azg():
            if taps == 9:
                _lib.check(L.azg_small_conv3x3(ctypes.c_void_p(xin.data_ptr()), *strides, B, H, pad,
                                               ctypes.c_void_p(wk.data_ptr()), cin, cout,
                                               ctypes.c_void_p(b.data_ptr()), 1, ctypes.c_void_p(y.data_ptr()), cout,
                                               st))
            else:
                _lib.check(L.azg_small_fc(ctypes.c_void_p(xin.data_ptr()), cin, B, ctypes.c_void_p(wk.data_ptr()),
                                          cin, cout, ctypes.c_void_p(b.data_ptr()), 1,
                                          ctypes.c_void_p(y.data_ptr()), cout, st))

        if taps == 9:
            xcl = x.contiguous(memory_format=torch.channels_last)

            def lib():
                torch.relu_(torch.nn.functional.conv2d(xcl, wk, b, padding=pad))
        else:
            xr = x.reshape(B, cin)

            def lib():
                torch.relu_(torch.addmm(b, xr, w.t()))
        for f in (azg, lib):
            for _ in range(5):
                f()
        ts = {"azg": [], "lib": []}
        for r in range(7):
            for k, f in (("azg", azg), ("lib", lib)) if r % 2 == 0 else (("lib", lib), ("azg", azg)):
                ts[k].append(timeit(f))
        print(json.dumps({"layer": name, "B": B, "azg_us": sorted(ts["azg"])[3],
                          "torch_us": sorted(ts["lib"])[3]}), flush=True)


if __name__ == "__main__":
    main()
