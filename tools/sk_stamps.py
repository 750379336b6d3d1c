"""Where a one-leaf split-K convolution's time goes: per-block wall-clock stamps (tools/Makefile
libazg_small_timing.so, azg_small.hip built with -DAZG_SMALL_TIMING) of conv3 (7x7 -> 5x5, 512 -> 512,
512 blocks) and conv12 (conv1 + conv2, 256 blocks) at one leaf, with the weights hot in L2 (back-to-back
launches), after a 64 MB sweep (past the L2s, not the MALL: the drop-in's case, the other layers' ~50 MB of
weights in between) and after a 512 MB sweep (from HBM).
Phases per block: 0 entry, 1 staged (input + weights in LDS), 2 products summed in LDS, 3 partials
stored and drained, 4 ticket taken, 5 (last block of a group) combined and stored.

    python tools/sk_stamps.py > gpurun_out/sk_stamps.json
"""
import ctypes
import json
import os

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    L = ctypes.CDLL(os.path.join(HERE, "libazg_small_timing.so"))
    P, I, I64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
    L.azg_small_conv3x3.argtypes = [P, I64, I, I, I, I, I, I, P, I, I, P, I, P, I, P, I64, P, I, P]
    L.azg_small_conv12.argtypes = [P, I, I, I, P, P, P, P, I, P, I, P, I64, P, I, P]
    L.azg_sk_stamps_read.argtypes = [P, I, P]
    V = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(0)
    C = 512
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    work = torch.zeros(8 * C * 64, device=dev)
    tickets = torch.zeros(C // 8 + 8, dtype=torch.int32, device=dev)
    sweep = torch.empty(128 * 1024 * 1024, device=dev)  # 512 MB
    x3 = torch.rand((1, 7, 7, C), generator=g).to(dev)
    w3 = (torch.randn((C, 3, 3, C), generator=g) * 0.02).to(dev)
    b3 = torch.randn((C,), generator=g).to(dev)
    y3 = torch.empty((25, C), device=dev)
    planes = (torch.rand((1, 4, 7, 7), generator=g) < 0.3).float().to(dev)
    w1 = (torch.randn((C, 3, 3, 4), generator=g) * 0.2).to(dev)
    b1 = torch.randn((C,), generator=g).to(dev)
    w2 = (torch.randn((C, 3, 3, C), generator=g) * 0.02).to(dev)
    y2 = torch.empty((49, C), device=dev)

    def conv3():
        assert L.azg_small_conv3x3(V(x3), 49 * C, 7 * C, C, 1, 1, 7, 0, V(w3), C, C, V(b3), 1, V(y3), C, V(work),
                                   work.numel(), V(tickets), tickets.numel(), st) == 0

    def conv12():
        assert L.azg_small_conv12(V(planes), 1, 4, 7, V(w1), V(b1), V(w2), V(b2), C, V(y2), C, V(work), work.numel(),
                                  V(tickets), tickets.numel(), st) == 0
    b2 = b1
    out = {}
    for name, fn, nblk in (("conv3", conv3, 512), ("conv12", conv12, 256)):
        for mode in ("hot", "l2swept", "swept"):
            runs = []
            for rep in range(12):
                if mode == "swept":  # past the L2s and the 256 MB MALL
                    sweep.add_(1.0)
                elif mode == "l2swept":  # 64 MB: past the eight 4 MB L2s, not the MALL
                    sweep[:16 * 1024 * 1024].add_(1.0)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn()
                e1.record()
                torch.cuda.synchronize()
                buf = (ctypes.c_ulonglong * (nblk * 8))()
                khz = ctypes.c_int32()
                assert L.azg_sk_stamps_read(ctypes.cast(buf, P), nblk * 8, ctypes.cast(ctypes.byref(khz), P)) == 0
                t = np.array(buf, dtype=np.float64).reshape(nblk, 8) * 1e3 / khz.value  # us
                if rep < 2:
                    continue
                t0 = t[:, 0].min()
                last = t[:, 5] >= t[:, 4]  # (a stamp 5 older than this launch's stamp 4 is stale)
                ph = {"start_spread": float(t[:, 0].max() - t0),
                      "stage": float(np.median(t[:, 1] - t[:, 0])), "stage_max": float((t[:, 1] - t[:, 0]).max()),
                      "compute": float(np.median(t[:, 2] - t[:, 1])),
                      "store_drain": float(np.median(t[:, 3] - t[:, 2])),
                      "store_drain_max": float((t[:, 3] - t[:, 2]).max()),
                      "ticket": float(np.median(t[:, 4] - t[:, 3])), "ticket_max": float((t[:, 4] - t[:, 3]).max()),
                      "combine": float(np.median((t[:, 5] - t[:, 4])[last])) if last.any() else None,
                      "end_last_block": float(t[:, 5].max() - t0) if last.any() else None,
                      "end_of_ticket": float(t[:, 4].max() - t0),
                      "event_us": e0.elapsed_time(e1) * 1e3}
                runs.append(ph)
            med = {k: float(np.median([r[k] for r in runs if r[k] is not None])) for k in runs[0]}
            out[f"{name}_{mode}"] = {k: round(v, 2) for k, v in med.items()}
            print(name, mode, out[f"{name}_{mode}"], flush=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
