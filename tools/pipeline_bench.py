"""Measure the hot path's consumers on one GPU.

  examples  azg_examples over the records of G full self-play games (stub
            evaluator, so the records are produced in seconds): replay +
            symmetry forms + labels, the reference's maxlenOfQueue window and
            the whole iteration; HBM-bound, 4 * (planes*cells + A + 1) bytes
            written per example.
  train     NNetWrapper.train_examples (512 channels, batch 512, Adam) on a
            device ExampleSet: examples/s and TFLOP/s (3 x 404.3 MFLOP per
            example for forward + backward).
  arena     BatchedArena, MCTSPlayer (random-init 512-channel net, 25 sims)
            against RandomPlayer and GreedyPlayer, args.arenaCompare = 40.
  host      the host restatement of Coach.py:74-90 (examples_from_record)
            on the same records, for scale.

    python tools/pipeline_bench.py [--games 4096] [--out gpurun_out/pipeline.json]
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
from azg_amd.examples import engine_examples  # noqa: E402


class Args(dict):
    __getattr__ = dict.__getitem__


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    best = None
    for _ in range(reps):
        t0 = time.perf_counter()
        out = fn()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    return best, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--games", type=int, default=4096)
    ap.add_argument("--train-batches", type=int, default=40)
    ap.add_argument("--arena-games", type=int, default=40)
    ap.add_argument("--out", default="gpurun_out/pipeline.json")
    a = ap.parse_args()
    res = {"device": torch.cuda.get_device_name(0)}

    # ---- records of full games
    t0 = time.perf_counter()
    eng = SelfPlayEngine(a.games, sims=25, max_turns=343, evaluator="stub")
    eng.play()
    torch.cuda.synchronize()
    res["records"] = {"games": a.games, "seconds": time.perf_counter() - t0,
                      "moves": int(eng.read_moves(counts=False)["moves"].sum())}
    print("records", res["records"], flush=True)

    # ---- examples
    per_ex = 4 * (4 * 49 + 343 + 1)
    ex_res = {}
    for label, maxlen in (("maxlenOfQueue_200000", 200000), ("whole_iteration", 36 * res["records"]["moves"])):
        if maxlen * per_ex > 60e9:
            maxlen = int(60e9 // per_ex)
            label = f"window_{maxlen}"
        dt, ex = timed(lambda: engine_examples(eng, 30, "reference", maxlen))
        n = len(ex)
        ex_res[label] = {"examples": n, "ms": dt * 1e3, "examples_per_s": n / dt,
                         "GB_written_per_s": n * per_ex / dt / 1e9, "bytes_per_example": per_ex}
        print("examples", label, ex_res[label], flush=True)
        del ex
        torch.cuda.empty_cache()
    res["examples"] = ex_res

    # ---- host restatement for scale (one game)
    from azg_amd.coach import examples_from_record
    from azg_amd.inflexion import InflexionGame
    rec = eng.read_moves()
    game = InflexionGame(7, max_turns=343, max_power=6)
    t0 = time.perf_counter()
    hx = examples_from_record(game, rec["actions"][0], rec["temps"][0], rec["counts"][0], int(rec["moves"][0]))
    dt = time.perf_counter() - t0
    res["host_examples"] = {"examples": len(hx), "seconds": dt, "examples_per_s": len(hx) / dt, "cores": 1,
                            "sample": "game 0 of the same records, Python restatement of Coach.py:74-90"}
    print("host", res["host_examples"], flush=True)
    eng.close()

    # ---- trainer
    from azg_amd.examples import ExampleSet
    from azg_amd.nnet import NNetWrapper
    torch.manual_seed(0)
    w = NNetWrapper(game, dict(epochs=1, batch_size=512), device="cuda")
    E = 512 * a.train_batches
    g = torch.Generator(device="cpu").manual_seed(1)
    exs = ExampleSet((torch.rand((E, 4, 7, 7), generator=g) < 0.3).float().cuda(),
                     torch.softmax(torch.randn((E, 343), generator=g), 1).cuda(),
                     (torch.randint(0, 2, (E,), generator=g).float() * 2 - 1).cuda())
    np.random.seed(0)
    w.train_examples(ExampleSet(exs.planes[:1024], exs.pis[:1024], exs.vs[:1024]))  # warm up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    losses = w.train_examples(exs)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    res["train"] = {"examples": E, "batch": 512, "seconds": dt, "examples_per_s": E / dt,
                    "TFLOP_per_s": E * 3 * 404.3e6 / dt / 1e12, "final_losses": losses[-1].tolist()}
    print("train", res["train"], flush=True)

    # ---- arena
    from azg_amd.arena import BatchedArena
    args = Args(numMCTSSims=25, cpuct=1)
    ar = {}
    for opp in ("random", "greedy"):
        arena = BatchedArena(game, w, args, opponent=opp)
        t0 = time.perf_counter()
        one, two, draws = arena.playGames(a.arena_games)
        dt = time.perf_counter() - t0
        ar[opp] = {"games": a.arena_games, "seconds": dt, "games_per_s": a.arena_games / dt,
                   "new_wins": one, "baseline_wins": two, "draws": draws}
        print("arena", opp, ar[opp], flush=True)
    res["arena"] = ar
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
