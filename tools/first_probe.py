"""winograd_first_kernel's write path in other shapes (tools/first_probe.hip), timed alone at
4096 leaves with HIP events, round-robin over the variants, each variant's V checked
bitwise against the product kernel's.  Prints one JSON line.

    make -C tools libfirst_probe.so && python tools/first_probe.py
"""
import ctypes
import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
NAMES = {0: "product", 1: "S0 wpb1", 2: "S1 wpb1", 3: "S0 wpb4", 4: "S1 wpb4", 5: "S0 wpb8", 6: "S1 wpb8",
         7: "S0 persist", 8: "S1 persist", 9: "S1 wpb4 persist", 10: "S1 wpb1 no-nt", 11: "S0 wpb1 no-nt",
         12: "S0 tile rows over 2 waves", 13: "S1 tile rows over 2 waves",
         14: "S0 rows/2 waves, wpb4", 15: "S0 one tile per wave", 16: "S0 one tile per wave, wpb4",
         17: "S0 rows/2 waves, wpb2"}


def planes_like_leaves(B, n, gen):
    """Inflexion leaf planes (InflexionGame.to_planes): own / opponent 0-1 planes (disjoint),
    constant turn and can-spawn planes."""
    own = (torch.rand(B, n, n, generator=gen) < 0.25)
    opp = (torch.rand(B, n, n, generator=gen) < 0.25) & ~own
    turn = torch.randint(0, 343, (B, 1, 1), generator=gen).expand(B, n, n)
    spawn = torch.randint(0, 2, (B, 1, 1), generator=gen).expand(B, n, n)
    return torch.stack([own.float(), opp.float(), turn.float(), spawn.float()], 1).contiguous()


def main():
    for B in [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "4096,256").split(",")]:
        probe(B)


def probe(B):
    L = ctypes.CDLL(os.path.join(HERE, "libfirst_probe.so"))
    L.first_probe.restype = ctypes.c_int
    vp, i32 = ctypes.c_void_p, ctypes.c_int
    L.first_probe.argtypes = [i32, vp, vp, vp, vp, i32, i32, i32, vp, i32, vp]
    n, C, depth = 7, 512, 4
    gen = torch.Generator().manual_seed(0)
    planes = planes_like_leaves(B, n, gen).cuda()
    w1 = (torch.randn(C, depth, 3, 3, generator=gen) * 0.05).cuda()
    b1 = (torch.randn(C, generator=gen) * 0.05).cuda()
    V = torch.empty(B * 121 * 2 * C, dtype=torch.int16, device="cuda")
    ovf = torch.zeros(1, dtype=torch.int32, device="cuda")
    st = vp(torch.cuda.current_stream().cuda_stream)
    variants = [int(v) for v in os.environ.get("VARIANTS", "0,1,3,5,12,14,15,16,17").split(",")]
    grid_waves = int(os.environ.get("GRID_WAVES", 0))

    def run(v):
        rc = L.first_probe(v, vp(planes.data_ptr()), vp(w1.data_ptr()), vp(b1.data_ptr()), vp(V.data_ptr()), B,
                           depth, C, vp(ovf.data_ptr()), grid_waves, st)
        if rc:
            raise RuntimeError(f"first_probe({v}) = {rc}")

    run(0)
    ref = V.clone()
    same = {}
    for v in variants:
        V.fill_(0)
        run(v)
        torch.cuda.synchronize()
        same[v] = bool(torch.equal(V, ref))
    del ref
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    times = {v: [] for v in variants}
    for _ in range(int(os.environ.get("ROUNDS", 9 if B >= 1024 else 41))):
        for v in variants:
            run(v)
            ev[0].record()
            run(v)
            ev[1].record()
            ev[1].synchronize()
            times[v].append(ev[0].elapsed_time(ev[1]) * 1e3)
    nbytes = V.numel() * 2
    out = {}
    for v in variants:
        t = sorted(times[v])
        med = t[len(t) // 2]
        out[NAMES.get(v, str(v))] = {"variant": v, "us_median": round(med, 1), "us_min": round(t[0], 1),
                                     "tb_s": round(nbytes / med / 1e6, 3), "bitwise_equal": same[v]}
    print(json.dumps({"batch": B, "bytes_written": nbytes, "grid_waves": grid_waves or 4096,
                      "overflow": int(ovf.item()), "variants": out}), flush=True)


if __name__ == "__main__":
    sys.exit(main())
