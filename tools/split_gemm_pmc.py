"""Run libazg's split GEMM on conv2's shape (4096 leaves) a fixed number of times, for
rocprofv3 --pmc passes on that kernel alone:

    rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES ... -- python3 tools/split_gemm_pmc.py <variant> [reps]
    python tools/split_gemm_pmc.py --summary <counter_collection.csv>...   (medians per counter)
"""
import csv
import ctypes
import json
import os
import sys
from collections import defaultdict


def run(variant, reps):
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import azg_amd  # noqa: F401
    from azg_amd import _lib
    from split_gemm_bench import layer_runs
    C = K = 512
    runs = layer_runs(7)  # conv2
    P = sum(p for p, _ in runs)
    rows = sum(p * t for p, t in runs)
    A = torch.randn(rows, 2 * C, device="cuda").half()
    Bt = torch.randn(P, K, 2 * C, device="cuda").half()
    M = torch.empty(rows * K, device="cuda")
    pts = (ctypes.c_int32 * len(runs))(*[p for p, _ in runs])
    rws = (ctypes.c_int32 * len(runs))(*[t for _, t in runs])
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    L = _lib.probes()
    for _ in range(reps):
        _lib.check(L.azg_split_gemm_variant(variant, ctypes.c_void_p(A.data_ptr()), ctypes.c_void_p(Bt.data_ptr()),
                                            ctypes.c_void_p(M.data_ptr()), len(runs), pts, rws, C, K, st))
    torch.cuda.synchronize()


def summary(paths):
    vals = defaultdict(list)
    for p in paths:
        for r in csv.DictReader(open(p)):
            if "split_gemm" in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {k: sorted(v)[len(v) // 2] for k, v in vals.items()}
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    if sys.argv[1] == "--summary":
        summary(sys.argv[2:])
    else:
        run(int(sys.argv[1]), int(sys.argv[2]) if len(sys.argv) > 2 else 10)
