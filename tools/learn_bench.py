"""One measured iteration of Coach.learn (Coach.py:92-165) on one MI355X at main.py's arguments
(main.py:14-33: numEps per GPU as configs[3], 25 sims, tempThreshold 30, maxlenOfQueue 200,000,
10 epochs of len/512 batches, NNet.py:13-22's 512-channel network), the phases timed apart:
self-play of numEps games + the example window (azg_examples on the GPU), training
(NNetWrapper.train_examples), the checkpoint write.  DESIGN.md 6's iteration-time split is
estimated from per-phase rates; this measures it.  Prints one JSON line.

    python tools/learn_bench.py [--eps 4096] [--epochs 10] [--iters 1]
"""
import argparse
import json
import os
import sys
import tempfile
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import azg_amd  # noqa: E402,F401
from azg_amd.coach import Coach  # noqa: E402
from azg_amd.inflexion import InflexionGame  # noqa: E402
from azg_amd.nnet import NNetWrapper  # noqa: E402


class Args(dict):
    __getattr__ = dict.__getitem__


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--eps", type=int, default=4096)
    ap.add_argument("--epochs", type=int, default=10)
    ap.add_argument("--iters", type=int, default=1)
    a = ap.parse_args()
    tmp = tempfile.mkdtemp(prefix="azg_learn_")
    args = Args(numIters=a.iters, numEps=a.eps, tempThreshold=30, updateThreshold=0.6, maxlenOfQueue=200000,
                numMCTSSims=25, arenaCompare=40, cpuct=1, checkpoint=tmp, load_model=False,
                load_folder_file=(tmp, "best.pth.tar"), numItersForTrainExamplesHistory=20, saveExamples=False)
    game = InflexionGame(7, max_turns=343, max_power=6)
    torch.manual_seed(0)
    nnet = NNetWrapper(game, dict(epochs=a.epochs), device="cuda")
    c = Coach(game, nnet, args)
    times = {"selfplay_s": 0.0, "train_s": 0.0, "checkpoint_s": 0.0}
    counts = {}

    def timed(name, fn):
        def wrap(*x, **k):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            out = fn(*x, **k)
            torch.cuda.synchronize()
            times[name] += time.perf_counter() - t0
            print(f"# {name} {time.perf_counter() - t0:.1f}s", file=sys.stderr, flush=True)
            return out
        return wrap

    sp = c._selfplay_iteration

    def selfplay(*x, **k):
        ex = sp(*x, **k)
        counts["examples_in_window"] = len(ex) if ex is not None else 0
        return ex
    c._selfplay_iteration = timed("selfplay_s", selfplay)
    te = nnet.train_examples

    def train(ex, *x, **k):
        counts["train_examples"] = len(ex)
        return te(ex, *x, **k)
    nnet.train_examples = timed("train_s", train)
    nnet.save_checkpoint = timed("checkpoint_s", nnet.save_checkpoint)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    c.learn(pit=False)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    steps = a.epochs * (counts.get("train_examples", 0) // 512) * a.iters
    print(json.dumps({"what": "Coach.learn iteration(s), 1 GPU", "iters": a.iters, "eps": a.eps, "epochs": a.epochs,
                      "wall_s": wall, **times, **counts, "train_steps": steps,
                      "train_examples_per_s": steps * 512 / times["train_s"] if times["train_s"] else None,
                      "selfplay_games_per_s": a.eps * a.iters / times["selfplay_s"] if times["selfplay_s"] else None}),
          flush=True)


if __name__ == "__main__":
    main()
