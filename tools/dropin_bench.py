"""Per-call time of the drop-in MCTS.getActionProb (one game, numMCTSSims leaves one at
a time: the reference's own main.py arrangement, BASELINE configs[0]) for the
evaluator forms a user can hand it.  Prints one JSON line per form."""
import argparse
import json
import sys
import time
import os

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import azg_amd  # noqa: E402,F401
from azg_amd.inflexion import InflexionGame  # noqa: E402
from azg_amd.mcts import MCTS  # noqa: E402
from azg_amd.nnet import InferenceNet, NNetWrapper  # noqa: E402
from azg_amd.othello import OthelloGame  # noqa: E402


class Args(dict):
    __getattr__ = dict.__getitem__


def run(ev, game, sims, graph, moves, fast=True):
    args = Args(numMCTSSims=sims, cpuct=1, tempThreshold=15)
    np.random.seed(1)
    mcts = MCTS(ev, args, graph=graph, fast=fast)
    g = game.restarted()
    times = []
    for _ in range(moves):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        pi = mcts.getActionProb(g, temp=1)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
        g = g.to_next_state(int(np.random.choice(len(pi), p=pi)))
    return float(np.median(times[2:]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--game", default="othello6")
    ap.add_argument("--sims", type=int, default=25)
    ap.add_argument("--moves", type=int, default=12)
    ap.add_argument("--forms", default="module,module-graph,default,library,small")
    a = ap.parse_args()
    game = OthelloGame(6) if a.game == "othello6" else OthelloGame(8) if a.game == "othello8" else \
        InflexionGame(7, max_turns=343, max_power=6)
    torch.manual_seed(0)
    w = NNetWrapper(game, device="cuda")
    for form in a.forms.replace("+", ",").split(","):  # ("+": tools/gpu.sh turns commas into spaces)
        fast = True
        if form.startswith("module"):  # the reference module itself (MCTS(fast=False))
            ev, graph, fast = w, form.endswith("graph"), False
        elif form == "default":  # MCTS's own default: the module's InferenceNet (small-batch kernels)
            ev, graph = w, True
        elif form == "library":  # BN folded, MIOpen / hipBLASLt at one leaf
            ev, graph = InferenceNet(w.nnet.eval(), conv="miopen", gemm="f32", small=False), True
        elif form == "layers":  # azg_small.hip one launch per layer (the default)
            ev, graph = InferenceNet(w.nnet.eval(), conv="miopen", gemm="f32", small=True), True
        else:  # "small": the probe library's one-launch forward (azg_small_net, tools/small_probes.py)
            import small_probes as sp
            ev, graph = sp.ProbeInferenceNet(w.nnet.eval(), conv="miopen", gemm="f32", small=True, mode="fused"), True
        t = run(ev, game, a.sims, graph, a.moves, fast)
        print(json.dumps({"game": a.game, "form": form, "sims": a.sims, "ms_per_call": t * 1e3,
                          "sims_per_s": a.sims / t}), flush=True)


if __name__ == "__main__":
    main()
