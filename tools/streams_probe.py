"""Probe: one configuration's games as K free-running engines on K HIP streams, each move
replayed from a captured HIP graph per engine (so the host issues K graph launches per
move, not K x ~400 kernel launches).  K = 1 is the bench's --graph arrangement.  Records
must not depend on K (game i is seeded by its global index): checked at the end.

    python tools/streams_probe.py --games 256 --ks 1,2,4 --moves 4 --rounds 5
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import azg_amd  # noqa: E402,F401
from azg_amd.engine import SelfPlayEngine  # noqa: E402
from azg_amd.nnet import InferenceNet, InflexionNNet  # noqa: E402


def build(net, G, K):
    streams = [torch.cuda.Stream() for _ in range(K)]
    engs = []
    for k, s in enumerate(streams):
        with torch.cuda.stream(s):
            e = SelfPlayEngine(G // K, sims=25, evaluator=InferenceNet(net), max_turns=343, first_game=k * (G // K))
            e.move()  # eager first move: libraries, workspaces
        engs.append(e)
    torch.cuda.synchronize()
    for e, s in zip(engs, streams):
        with torch.cuda.stream(s):
            e.capture_move()
    torch.cuda.synchronize()
    return engs, streams


class OneGraph:
    """The K engines' moves captured as ONE graph whose K branches are forked onto K streams
    inside the capture (event fork / join), so the graph itself carries the concurrency."""

    def __init__(self, engs, streams):
        self.engs, self.streams = engs, streams
        torch.cuda.synchronize()
        self.g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.g):
            main = torch.cuda.current_stream()
            for e, s in zip(engs, streams):
                s.wait_stream(main)
                with torch.cuda.stream(s):
                    for _ in range(e.sims):
                        e.simulate()
                    e.move_end()
            for s in streams:
                main.wait_stream(s)
        torch.cuda.synchronize()


def build_one_graph(net, G, K):
    streams = [torch.cuda.Stream() for _ in range(K)]
    engs = []
    for k, s in enumerate(streams):
        with torch.cuda.stream(s):
            e = SelfPlayEngine(G // K, sims=25, evaluator=InferenceNet(net), max_turns=343, first_game=k * (G // K))
            e.move()
        engs.append(e)
    torch.cuda.synchronize()
    return OneGraph(engs, streams), None


def timed(engs, streams, moves):
    if isinstance(engs, OneGraph):
        torch.cuda.synchronize()
        e0 = sum(e.stats()["expansions"] for e in engs.engs)
        t0 = time.perf_counter()
        for _ in range(moves):
            engs.g.replay()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        return (sum(e.stats()["expansions"] for e in engs.engs) - e0) / dt, dt / moves * 1e3
    torch.cuda.synchronize()
    e0 = sum(e.stats()["expansions"] for e in engs)
    t0 = time.perf_counter()
    for _ in range(moves):
        for e, s in zip(engs, streams):
            with torch.cuda.stream(s):
                e.move()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return (sum(e.stats()["expansions"] for e in engs) - e0) / dt, dt / moves * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--games", type=int, default=256)
    ap.add_argument("--ks", default="1,2,4")
    ap.add_argument("--moves", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    torch.manual_seed(0)
    net = InflexionNNet().cuda().eval()
    ks = [int(k) if not k.startswith("g") else k for k in a.ks.replace("/", ",").split(",")]
    arr = {k: (build(net, a.games, k) if isinstance(k, int) else build_one_graph(net, a.games, int(k[1:])))
           for k in ks}
    res = {}
    for r in range(a.rounds):
        for k in ks:
            v, ms = timed(*arr[k], a.moves)
            res.setdefault(k, []).append((v, ms))
        print(json.dumps({"round": r, **{f"k{k}": round(x[-1][0]) for k, x in res.items()}}), flush=True)
    # records of the first moves equal whatever K (same games, same seeds)
    recs = {}
    for k, (engs, _) in arr.items():
        if isinstance(engs, OneGraph):
            engs = engs.engs
        torch.cuda.synchronize()
        for e in engs:
            e.check_evaluator()
            assert e.stats()["error"] == 0
        rs = [e.read_moves() for e in engs]
        recs[k] = (np.concatenate([r["actions"] for r in rs]), np.concatenate([r["moves"] for r in rs]))
    k0 = ks[0]
    for k in ks[1:]:
        m = int(min(recs[k][1].min(), recs[k0][1].min()))
        print(json.dumps({"k": k, "records_equal_first_moves": m,
                          "equal": bool((recs[k][0][:, :m] == recs[k0][0][:, :m]).all())}), flush=True)
    for k, x in res.items():
        vs = sorted(v for v, _ in x)
        print(json.dumps({"k": k, "games": a.games, "median_exp_per_s": vs[len(vs) // 2], "min": vs[0],
                          "max": vs[-1], "ms_per_move": sorted(m for _, m in x)[len(x) // 2]}), flush=True)


if __name__ == "__main__":
    main()
