"""Time libazg's split GEMM (azg_split_gemm) on the leaf network's Winograd GEMM shapes
at 4096 leaves (AZG_SG_LEAVES), every kernel variant, against the same products as one hipBLASLt fp16
GEMM ([hi|lo|hi] rows) and the f32 GEMM; median (and best) of 7 round-robin rounds.
TF/s are of the executed fp16 MFMA work (3 products per f32 multiply-add).

    python tools/split_gemm_bench.py > gpurun_out/split_gemm_bench.json
"""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import azg_amd  # noqa: E402,F401
from azg_amd import _lib  # noqa: E402

# AZG_SG_VARIANTS="4,6,15,16" times the probes instead (6/15/16 give wrong results by design)
VARIANTS = tuple(int(v) for v in os.environ.get("AZG_SG_VARIANTS", "0,4,7,12").split(","))


def layer_runs(h_out, B=4096):
    """(points, rows) runs of one layer's GEMMs as InferenceNet._winograd_gemms forms them."""
    from azg_amd.nnet import winograd_groups
    runs = []
    for _, _, P, n in winograd_groups(h_out):
        if runs and runs[-1][1] == B * n:
            runs[-1][0] += P
        else:
            runs.append([P, B * n])
    return [tuple(r) for r in runs]


# AZG_SG_LEAVES=256 times the shapes of a 256-leaf forward (C2) instead of 4096
LEAVES = int(os.environ.get("AZG_SG_LEAVES", "4096"))
LAYERS = {"conv2": layer_runs(7, LEAVES), "conv3": layer_runs(5, LEAVES), "conv4": layer_runs(3, LEAVES)}


def timeit(fn, reps=10):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps


def time_all(fns, rounds=7):
    """Round-robin over the candidates (the order rotates per round) after a warm-up
    of every one, so clock ramps and box state do not favour whichever runs first;
    returns {name: (median ms, min ms)} over the rounds."""
    for _, fn in fns:
        for _ in range(5):
            fn()
    ms = {k: [] for k, _ in fns}
    for r in range(rounds):
        order = fns[r % len(fns):] + fns[:r % len(fns)]
        for k, fn in order:
            ms[k].append(timeit(fn))
    return {k: (sorted(v)[len(v) // 2], min(v)) for k, v in ms.items()}


def main():
    C = K = 512
    L = _lib.probes()
    out = []
    for name, runs in LAYERS.items():
        P = sum(p for p, _ in runs)
        rows = sum(p * t for p, t in runs)
        A = torch.randn(rows, 2 * C, device="cuda").half()
        Bt = torch.randn(P, K, 2 * C, device="cuda").half()
        M = torch.empty(rows * K, device="cuda")
        pts = (ctypes.c_int32 * len(runs))(*[p for p, _ in runs])
        rws = (ctypes.c_int32 * len(runs))(*[t for _, t in runs])
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

        def azg_variant(v):
            def fn():
                _lib.check(L.azg_split_gemm_variant(v, ctypes.c_void_p(A.data_ptr()), ctypes.c_void_p(Bt.data_ptr()),
                                                    ctypes.c_void_p(M.data_ptr()), len(runs), pts, rws, C, K, st))
            return fn

        A3 = torch.randn(rows, 3 * C, device="cuda").half()
        B3 = torch.randn(P, 3 * C, K, device="cuda").half()
        Vf = torch.randn(rows, C, device="cuda")
        Uf = torch.randn(P, C, K, device="cuda")

        def blas():
            r = pt = 0
            for p, t in runs:
                torch.bmm(A3[r:r + p * t].view(p, t, 3 * C), B3[pt:pt + p], out_dtype=torch.float32,
                          out=M[r * K:(r + p * t) * K].view(p, t, K))
                r += p * t
                pt += p

        def f32():
            r = pt = 0
            for p, t in runs:
                torch.bmm(Vf[r:r + p * t].view(p, t, C), Uf[pt:pt + p], out=M[r * K:(r + p * t) * K].view(p, t, K))
                r += p * t
                pt += p

        flops16 = 3 * 2.0 * rows * C * K
        row = {"layer": name, "runs": runs}
        def azg_default():
            _lib.check(L.azg_split_gemm(ctypes.c_void_p(A.data_ptr()), ctypes.c_void_p(Bt.data_ptr()),
                                        ctypes.c_void_p(M.data_ptr()), len(runs), pts, rws, C, K, st))

        fns = [("azg_v%d" % v, azg_variant(v)) for v in VARIANTS] + [("azg_default", azg_default), ("hipblaslt_split", blas),
                                                                         ("hipblaslt_f32", f32)]
        for k, (med, mn) in time_all(fns).items():
            fl = flops16 if k != "hipblaslt_f32" else flops16 / 3
            row[k + "_ms"] = med
            row[k + "_tflops"] = fl / med / 1e9
            row[k + "_best_tflops"] = fl / mn / 1e9
        print(json.dumps(row), flush=True)
        out.append(row)
        del A, Bt, M, A3, B3, Vf, Uf
        torch.cuda.empty_cache()
    return out


if __name__ == "__main__":
    main()
