"""Probe: f32 throughput of the leaf network on the GPU in several layouts."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from azg_amd.nnet import InflexionNNet  # noqa: E402

FLOP_PER_LEAF = 404.3e6


def bench(fn, x, iters=10):
    for _ in range(3):
        fn(x)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn(x)
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


def main():
    torch.manual_seed(0)
    net = InflexionNNet().cuda().eval()
    res = {}
    for B in [256, 1024, 4096]:
        x = torch.randint(0, 2, (B, 4, 7, 7), device="cuda").float()
        with torch.no_grad():
            for name, mod, xx, dt in [
                ("nchw_f32", net, x, None),
                ("cl_f32", net.to(memory_format=torch.channels_last), x.to(memory_format=torch.channels_last), None),
                ("nchw_bf16", net, x, torch.bfloat16),
            ]:
                if dt is None:
                    f = lambda z, m=mod: m(z)
                else:
                    f = lambda z, m=mod, d=dt: torch.autocast("cuda", dtype=d)(m)(z)
                s = bench(f, xx)
                res[f"{name}_B{B}"] = {"ms": s * 1e3, "tflops": B * FLOP_PER_LEAF / s / 1e12}
                print(name, B, f"{s*1e3:.3f} ms", f"{B*FLOP_PER_LEAF/s/1e12:.1f} TF/s", flush=True)
            net = net.to(memory_format=torch.contiguous_format)
    json.dump(res, open("gpurun_out/nn_probe.json", "w"), indent=1)


if __name__ == "__main__":
    main()
