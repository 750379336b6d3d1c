"""Measured iteration(s) of Coach.learn (Coach.py:92-165) on one MI355X at main.py's arguments
(main.py:14-33: numEps per GPU as configs[3], 25 sims, tempThreshold 30, maxlenOfQueue 200,000,
numItersForTrainExamplesHistory 20, 10 epochs of len/512 batches, NNet.py:13-22's 512-channel
network), the phases timed apart: self-play of numEps games + the example window (azg_examples
on the GPU), the examples file (saveTrainExamples), the shuffle (Coach.py:149), training
(NNetWrapper.train_examples), the checkpoint write.  Prints one JSON line.

    python tools/learn_bench.py [--eps 4096] [--epochs 10] [--iters 1] [--steady]

--steady measures the loop's steady state instead of its first iteration: the history already
holds numItersForTrainExamplesHistory - 1 earlier windows (this iteration's window reused as
their content, already saved by "earlier iterations" -- set up untimed), so the timed iteration
appends its window, saves the examples file (one new window written), shuffles and trains on
all 20 windows (4M examples x 10 epochs at 4096 games per iteration), as every iteration after
the 20th does.  Host RSS (current and peak) and device memory are reported.
"""
import argparse
import json
import os
import resource
import sys
import tempfile
import time

import psutil
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import azg_amd  # noqa: E402,F401
import azg_amd.examples as azg_examples  # noqa: E402
from azg_amd.coach import Coach  # noqa: E402
from azg_amd.examples import ExampleSet, save_window  # noqa: E402
from azg_amd.inflexion import InflexionGame  # noqa: E402
from azg_amd.nnet import NNetWrapper  # noqa: E402


class Args(dict):
    __getattr__ = dict.__getitem__


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--eps", type=int, default=4096)
    ap.add_argument("--epochs", type=int, default=10)
    ap.add_argument("--iters", type=int, default=1)
    ap.add_argument("--history", type=int, default=20, help="numItersForTrainExamplesHistory (main.py:27)")
    ap.add_argument("--steady", action="store_true", help="the history full before the timed iteration")
    ap.add_argument("--save", choices=["azg", "reference", "off"], default="azg", help="examples file format")
    a = ap.parse_args()
    tmp = tempfile.mkdtemp(prefix="azg_learn_")
    args = Args(numIters=a.iters, numEps=a.eps, tempThreshold=30, updateThreshold=0.6, maxlenOfQueue=200000,
                numMCTSSims=25, arenaCompare=40, cpuct=1, checkpoint=tmp, load_model=False,
                load_folder_file=(tmp, "best.pth.tar"), numItersForTrainExamplesHistory=a.history,
                saveExamples=a.save != "off", examplesFormat=a.save if a.save != "off" else "azg")
    game = InflexionGame(7, max_turns=343, max_power=6)
    torch.manual_seed(0)
    nnet = NNetWrapper(game, dict(epochs=a.epochs), device="cuda")
    c = Coach(game, nnet, args)
    times = {"selfplay_s": 0.0, "save_examples_s": 0.0, "shuffle_s": 0.0, "train_s": 0.0, "checkpoint_s": 0.0,
             "setup_untimed_s": 0.0}
    counts = {}

    def timed(name, fn):
        def wrap(*x, **k):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            out = fn(*x, **k)
            torch.cuda.synchronize()
            times[name] += time.perf_counter() - t0
            print(f"# {name} {time.perf_counter() - t0:.2f}s rss {psutil.Process().memory_info().rss / 2**30:.1f} GiB",
                  file=sys.stderr, flush=True)
            return out
        return wrap

    sp = c._selfplay_iteration

    def selfplay(*x, **k):
        ex = sp(*x, **k)
        counts["examples_in_window"] = len(ex) if ex is not None else 0
        return ex
    timed_sp = timed("selfplay_s", selfplay)

    def selfplay_then_fill(*x, **k):
        ex = timed_sp(*x, **k)
        if a.steady and not c.trainExamplesHistory:
            # untimed set-up: history - 1 earlier windows (this window's content, one file saved
            # once as the earlier iterations would have), so the timed save writes one window
            t0 = time.perf_counter()
            path = os.path.join(tmp, "earlier_window.npz")
            if a.save == "azg":
                save_window(ex, path)
            c.trainExamplesHistory = []
            for _ in range(a.history - 1):
                w = ExampleSet(ex.planes, ex.pis, ex.vs)
                if a.save == "azg":
                    w.saved_path = path
                c.trainExamplesHistory.append(w)
            torch.cuda.synchronize()
            times["setup_untimed_s"] += time.perf_counter() - t0
        return ex
    c._selfplay_iteration = selfplay_then_fill
    c.saveTrainExamples = timed("save_examples_s", c.saveTrainExamples)
    azg_examples.shuffle_perm = timed("shuffle_s", azg_examples.shuffle_perm)
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
    wall = time.perf_counter() - t0 - times["setup_untimed_s"]
    steps = a.epochs * (counts.get("train_examples", 0) // 512) * a.iters
    window_bytes = 0
    wdir = os.path.join(tmp, "examples_windows")
    if os.path.isdir(wdir):
        window_bytes = max(os.path.getsize(os.path.join(wdir, f)) for f in os.listdir(wdir))
    other = wall - sum(v for k, v in times.items() if k != "setup_untimed_s")
    print(json.dumps({"what": "Coach.learn iteration(s), 1 GPU" + (", steady state (history full)" if a.steady else ""),
                      "iters": a.iters, "eps": a.eps, "epochs": a.epochs, "history_windows": a.history,
                      "examples_format": a.save,
                      "wall_s": wall, **times, "cat_index_other_s": other, **counts, "train_steps": steps,
                      "train_ms_per_step": times["train_s"] / steps * 1e3 if steps else None,
                      "train_examples_per_s": steps * 512 / times["train_s"] if times["train_s"] else None,
                      "selfplay_games_per_s": a.eps * a.iters / times["selfplay_s"] if times["selfplay_s"] else None,
                      "saved_window_bytes": window_bytes,
                      "host_rss_gib": psutil.Process().memory_info().rss / 2 ** 30,
                      "host_peak_rss_gib": resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 2 ** 20,
                      "device_peak_gib": torch.cuda.max_memory_allocated() / 2 ** 30}),
          flush=True)


if __name__ == "__main__":
    main()
