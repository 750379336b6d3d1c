"""Probe: the Winograd GEMM batches as error-compensated fp16 (3 MFMA products per term).

Each f32 operand x is split exactly as x = hi + lo + r, hi = fp16(x), lo = fp16(x - hi),
|r| <= 2^-22 |x| (normal range).  hi*hi + hi*lo + lo*hi is then the f32 product to about
2^-21 relative, and the MFMA accumulates in f32.  One GEMM computes it with the split
written along K: A' = [a_hi | a_lo | a_hi] (T x 3C), B' = [b_hi ; b_hi ; b_lo] (3C x K).

Times f32 torch.bmm against the split form (and a two-call variant) for conv2-4's shapes
at 4096 leaves and prints the error of both against an f64 product.

    python tools/split_gemm_probe.py > gpurun_out/split_gemm_probe.json
"""
import json
import sys

import torch


def split16(x):
    hi = x.half()
    lo = (x - hi.float()).half()
    return hi, lo


def timeit(fn, reps=10):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps


def main():
    dev = "cuda"
    torch.manual_seed(0)
    E, C, K = 25, 512, 512
    out = []
    for name, T in (("conv2", 4096 * 9), ("conv3", 4096 * 4), ("conv4", 4096)):
        V = (torch.randn(E, T, C, device=dev) * 2.0).relu_() - 0.3
        U = (torch.rand(E, C, K, device=dev) - 0.5) * 0.06
        scale = 2.0 ** 12  # power of two: keeps U's low halves out of fp16 subnormals
        Us = U * scale
        vh, vl = split16(V)
        uh, ul = split16(Us)
        A3 = torch.cat([vh, vl, vh], dim=2).contiguous()
        B3 = torch.cat([uh, uh, ul], dim=1).contiguous()
        A2 = torch.cat([vh, vl], dim=2).contiguous()
        B2 = torch.cat([uh, uh], dim=1).contiguous()
        M32 = torch.empty(E, T, K, device=dev)
        flops = 2.0 * E * T * C * K

        def f32():
            torch.bmm(V, U, out=M32)

        def s3():
            return torch.bmm(A3, B3, out_dtype=torch.float32)

        def s2():
            m = torch.bmm(A2, B2, out_dtype=torch.float32)
            return torch.baddbmm(m, A2[:, :, :C], ul, out_dtype=torch.float32)

        t32, t3, t2 = timeit(f32), timeit(s3), timeit(s2)
        # accuracy on a slice against f64
        ref = torch.bmm(V[:2].double(), U[:2].double())
        f32()
        e32 = (M32[:2].double() - ref).abs()
        m3 = s3()[:2].double() / scale
        e3 = (m3 - ref).abs()
        m2 = s2()[:2].double() / scale
        e2 = (m2 - ref).abs()
        rms = ref.pow(2).mean().sqrt().item()
        row = dict(layer=name, T=T, f32_ms=t32, f32_tflops=flops / t32 / 1e9,
                   split3_ms=t3, split3_eff_tflops=flops / t3 / 1e9,
                   split2_ms=t2, split2_eff_tflops=flops / t2 / 1e9,
                   rms=rms, err_f32_max=e32.max().item() / rms, err_split3_max=e3.max().item() / rms,
                   err_split2_max=e2.max().item() / rms,
                   err_f32_rms=e32.pow(2).mean().sqrt().item() / rms,
                   err_split3_rms=e3.pow(2).mean().sqrt().item() / rms)
        print(json.dumps(row), flush=True)
        out.append(row)
        del V, U, Us, vh, vl, uh, ul, A3, B3, A2, B2, M32
        torch.cuda.empty_cache()
    return out


if __name__ == "__main__":
    sys.exit(0 if main() else 1)
