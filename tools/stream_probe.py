"""Probe: does splitting the leaf batch over HIP streams overlap the Winograd
transforms / FC layers (HBM-bound) of one chunk with the GEMMs (MFMA-bound) of
another?  Times InferenceNet forwards at 4096 leaves: one stream, and k chunks
on k streams (each chunk's forward starts once the previous chunk's conv2 input
transform has been issued... approximated by a fixed event after its conv1)."""
import sys
import time

import torch

sys.path.insert(0, ".")
import azg_amd  # noqa: E402,F401
from azg_amd.nnet import InferenceNet, InflexionNNet  # noqa: E402


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / it


def main():
    torch.manual_seed(0)
    B = 4096
    net = InflexionNNet().cuda().eval()
    x = (torch.rand(B, 4, 7, 7, device="cuda") < 0.3).float()
    base = InferenceNet(net, conv="winograd").cuda()
    with torch.no_grad():
        t1 = timeit(lambda: base(x))
        print(f"1 stream: {t1 * 1e3:.3f} ms", flush=True)
        for k in (2, 4):
            nets = [InferenceNet(net, conv="winograd").cuda() for _ in range(k)]  # own workspaces
            streams = [torch.cuda.Stream() for _ in range(k)]
            xs = x.chunk(k)

            def run():
                cur = torch.cuda.current_stream()
                outs = []
                prev = None
                for j in range(k):
                    s = streams[j]
                    s.wait_stream(cur)
                    if prev is not None:
                        s.wait_event(prev)
                    with torch.cuda.stream(s):
                        ev = torch.cuda.Event()
                        hook_fired = []

                        def hook(i, what, ev=ev, hook_fired=hook_fired):
                            if i == 2 and what == "stop" and not hook_fired:
                                ev.record()
                                hook_fired.append(1)
                        nets[j].conv_hook = hook
                        outs.append(nets[j](xs[j]))
                        prev = ev
                for s in streams:
                    cur.wait_stream(s)
                return torch.cat([o[0] for o in outs]), torch.cat([o[1] for o in outs])
            tk = timeit(run)
            print(f"{k} streams (staggered by one conv2): {tk * 1e3:.3f} ms ({t1 / tk:.3f}x)", flush=True)


if __name__ == "__main__":
    main()
