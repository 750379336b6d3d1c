"""Where a split-GEMM stage spends its cycles: the diagnostic stamp build
(azg_split_gemm_stamps) on conv2's shape at 4096 leaves; prints the share of each
segment per wave (median over waves) -- shares, not run time (the stamps' waits
forbid overlaps the real kernel has).

    python tools/split_gemm_stamps.py > gpurun_out/stamps.json
"""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import azg_amd  # noqa: E402,F401
from azg_amd import _lib  # noqa: E402

SEGMENTS = ["reads+dma_issue (reads landed)", "mfma_issue", "vmcnt_wait", "barrier", "epilogue"]


def main():
    C = K = 512
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from split_gemm_bench import layer_runs
    runs = layer_runs(7)  # conv2
    P = sum(p for p, _ in runs)
    rows = sum(p * t for p, t in runs)
    A = torch.randn(rows, 2 * C, device="cuda").half()
    Bt = torch.randn(P, K, 2 * C, device="cuda").half()
    M = torch.empty(rows * K, device="cuda")
    cap = 1024 * 8 * 5
    st = torch.zeros(cap, dtype=torch.int64, device="cuda")
    pts = (ctypes.c_int32 * len(runs))(*[p for p, _ in runs])
    rws = (ctypes.c_int32 * len(runs))(*[t for _, t in runs])
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    L = _lib.probes()
    for _ in range(5):
        _lib.check(L.azg_split_gemm_stamps(ctypes.c_void_p(A.data_ptr()), ctypes.c_void_p(Bt.data_ptr()),
                                           ctypes.c_void_p(M.data_ptr()), len(runs), pts, rws, C, K,
                                           ctypes.c_void_p(st.data_ptr()), cap, s))
    torch.cuda.synchronize()
    blocks = min(256, torch.cuda.get_device_properties(0).multi_processor_count)
    v = st[:blocks * 8 * 5].view(blocks * 8, 5).double()
    tot = v.sum(1, keepdim=True)
    share = (v / tot).median(0).values.tolist()
    out = {"segments": SEGMENTS, "median_share": share, "median_cycles_per_wave": v.median(0).values.tolist(),
           "stages_per_wave": 16 * 5408 / blocks}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
