"""SelfPlayEngine.play() with the move captured as a HIP graph ("auto": batches up to GRAPH_MAX_GAMES)
against the eager loop, alternating, whole games, the random-init network's split form: node
expansions/s per arm.

    python tools/play_graph_ab.py [G] [sims]
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import azg_amd  # noqa: E402,F401
from azg_amd.engine import SelfPlayEngine  # noqa: E402
from azg_amd.nnet import InferenceNet, InflexionNNet  # noqa: E402


def main():
    G = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    sims = int(sys.argv[2]) if len(sys.argv) > 2 else 25
    torch.manual_seed(0)
    ev = InferenceNet(InflexionNNet().cuda().eval())
    e = SelfPlayEngine(G, sims=sims, evaluator=ev)
    e.play(max_moves=2, graph=False)  # warm up the kernels
    for rep in range(3):
        for graph in (False, "auto"):
            e.reset()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            moves = e.play(graph=graph)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            exp = e.stats()["expansions"] if "expansions" in e.stats() else None
            print(json.dumps({"G": G, "sims": sims, "graph": str(graph), "moves": moves, "seconds": dt,
                              "moves_per_s": moves / dt, "expansions": exp,
                              "expansions_per_s": exp / dt if exp else None}), flush=True)
    e.close()


if __name__ == "__main__":
    main()
