"""winograd_mid<7> (conv2 -> conv3) timed alone and right after a conv2-shaped split GEMM,
to tell a layout cost from the clock a preceding GEMM leaves behind (HISTORY.md 6b).

    python tools/mid_probe.py > gpurun_out/mid_probe.json
"""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import azg_amd  # noqa: E402,F401
from azg_amd import _lib  # noqa: E402


def main():
    L = _lib.lib()
    if os.environ.get("AZG_PROBE_LIB"):  # an alternative build of libazg (probe builds only)
        L = ctypes.CDLL(os.environ["AZG_PROBE_LIB"])
        for name, res, args in _lib.SIGNATURES:
            getattr(L, name).restype, getattr(L, name).argtypes = res, args
    C = K = 512
    B, H = 4096, 7
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from split_gemm_bench import layer_runs
    runs = layer_runs(7)  # conv2
    rows = sum(p * t for p, t in runs)
    P = sum(p for p, _ in runs)
    A = torch.randn(rows, 2 * C, device="cuda").half()
    Bt = torch.randn(P, K, 2 * C, device="cuda").half()
    M = torch.randn(rows * K, device="cuda")
    bias = torch.randn(K, device="cuda")
    V = torch.empty(B * 81 * 2 * K, device="cuda", dtype=torch.float16)
    ovf = torch.zeros(1, dtype=torch.int32, device="cuda")
    pts = (ctypes.c_int32 * 3)(*[p for p, _ in runs])
    rws = (ctypes.c_int32 * 3)(*[t for _, t in runs])
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    def gemm():
        _lib.check(L.azg_split_gemm(ctypes.c_void_p(A.data_ptr()), ctypes.c_void_p(Bt.data_ptr()),
                                    ctypes.c_void_p(M.data_ptr()), 3, pts, rws, C, K, st))

    def mid():
        _lib.check(L.azg_winograd_mid_nhwc(ctypes.c_void_p(M.data_ptr()), ctypes.c_void_p(bias.data_ptr()),
                                           ctypes.c_void_p(V.data_ptr()), B, H, K, 2.0 ** -10, 2,
                                           ctypes.c_void_p(ovf.data_ptr()), st))

    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    for _ in range(3):
        gemm()
        mid()
    alone, after, g = [], [], []
    for _ in range(10):
        torch.cuda.synchronize()
        ev[0].record()
        mid()
        ev[1].record()
        ev[1].synchronize()
        alone.append(ev[0].elapsed_time(ev[1]))
        torch.cuda.synchronize()
        ev[0].record()
        gemm()
        ev[1].record()
        mid()
        ev[2].record()
        ev[2].synchronize()
        g.append(ev[0].elapsed_time(ev[1]))
        after.append(ev[1].elapsed_time(ev[2]))
    med = lambda xs: sorted(xs)[len(xs) // 2] * 1000.0  # noqa: E731
    print(json.dumps({"lib": os.environ.get("AZG_PROBE_LIB", "libazg.so"), "mid7_alone_us": med(alone), "mid7_after_gemm_us": med(after), "gemm_us": med(g)}), flush=True)


if __name__ == "__main__":
    main()
