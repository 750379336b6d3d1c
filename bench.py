"""Self-play throughput of the MI355X engine (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C1..C5] [--games G] [--sims S]

One *step* = one move of every concurrent game: numMCTSSims simulations
(select -> leaf-batched network f32 forward -> expand/backup) followed by the
root-policy / sample / apply kernel -- the reference's Coach.executeEpisode
loop body (Coach.py:65-84) for G games at once.

Default workload (north_star target, configs[3] per GPU): 7x7 Inflexion,
max_turns 343, 4096 games per GPU, 25 sims/move, cpuct 1, tempThreshold 30,
random-init InflexionNNet (torch.manual_seed(0)), f32.  Presets: C1 6x6
Othello (1 game, 25 sims), C2 Inflexion 256 games x 25, C3 4096 x 100,
C4 4096/GPU x 25, C5 8x8 Othello 4096/GPU x 200.

`value` = node expansions per second over the whole job (new tree nodes =
network leaf evaluations, MCTS.py:89-112; terminal hits excluded), all ranks
summed.  Multi-GPU: one process per GPU (torchrun), games sharded by global
index, no communication inside self-play; each timed region ends with the
per-iteration RCCL example gather + weight broadcast (configs[3]).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

F32_MFMA_PEAK_TF = 157.3         # MI355X_MICROARCH.md: f32 matrix peak (dense)
F16_MFMA_PEAK_TF = 2500.0        # MI355X_MICROARCH.md: BF16/FP16 MFMA peak (dense)
HBM_PEAK_GBS = 8000.0            # MI355X_MICROARCH.md: HBM3E spec peak
EXPANSIONS_PER_GAME_REF = 8555   # reference random-init Inflexion episodes
GEMM_PMC_FILE = os.path.join(ROOT, "profiles", "r05_split_gemm_pmc_v4.json")  # the azg_split_gemm default (round 5 tree)
# PMC passes of the current Winograd tiling (F(4,3)+F(3,3) / F(5,3) / F(3,3)); the r01 files
# were measured on the earlier F(3,3)/F(2,3) tiling and are kept for the record only
PMC_FILE_WINOGRAD = {"split": os.path.join(ROOT, "profiles", "r06_pmc_C4.json")}  # (round 6 pass; r05 agrees to 1e-4)

PRESETS = {
    "C1": dict(game="othello", n=6, games=1, sims=25),
    "C2": dict(game="inflexion", n=7, games=256, sims=25),
    "C3": dict(game="inflexion", n=7, games=4096, sims=100),
    "C4": dict(game="inflexion", n=7, games=4096, sims=25),
    "C5": dict(game="othello", n=8, games=4096, sims=200),
}


def net_flops(n, depth, A, c=512):
    """FLOPs per leaf of InflexionNNet(n, depth, A, c): (whole forward, conv2+conv3+conv4).
    Inflexion 7x7: 404.3 M / 391.6 M."""
    conv1 = 2 * depth * c * 9 * n * n
    conv234 = 2 * c * c * 9 * (n * n + (n - 2) ** 2 + (n - 4) ** 2)
    fc = 2 * (c * (n - 4) ** 2 * 1024 + 1024 * 512 + 512 * A + 512)
    return conv1 + conv234 + fc, conv234


def transform_bytes(n, depth, c=512, split=True):
    """Algorithmic HBM bytes per leaf of the fused Winograd transforms (azg_winograd.hip),
    each operand read or written once at its stored width: winograd_first reads the planes
    and writes conv2's V; each winograd_mid reads layer i's M (f32) and writes layer i+1's
    V; winograd_out reads conv4's M and writes the flattened activation ([hi|lo|hi] fp16
    rows for fc1 in the split form, else f32).  V is 4 B per element (split hi + lo, or
    f32), M 4 B.  7x7 Inflexion, split: 0.247 + 0.348 + 0.151 + 0.079 = 0.826 MB."""
    from azg_amd.nnet import winograd_points
    h = [n, n - 2, n - 4]
    first = depth * n * n * 4 + winograd_points(h[0]) * c * 4
    mids = [winograd_points(h[i]) * c * 4 + winograd_points(h[i + 1]) * c * 4 for i in range(2)]
    out = winograd_points(h[2]) * c * 4 + h[2] * h[2] * c * (6 if split else 4)
    return {"first": first, "mid": sum(mids), "out": out, "total": first + sum(mids) + out}


def winograd_flops(n, c=512):
    """GEMM FLOPs per leaf of conv2-4 as mixed F(2..5,3) Winograd
    (nnet.winograd_points: (sum of tile sides + 2)^2 transformed points per image x 2 C K):
    7x7 board (11^2 + 7^2 + 5^2) x 2 x 512^2 = 102.2 M vs 391.6 M direct."""
    from azg_amd.nnet import winograd_points
    return sum(winograd_points(h) * 2 * c * c for h in (n, n - 2, n - 4))


# mean valid actions per visited node (87 for 7x7 Inflexion; legal
# moves of random-play Othello positions for the builder's plugin)
VALID_ACTIONS = {("inflexion", 7): 87.0, ("othello", 6): 6.0, ("othello", 8): 9.0}


def tree_bytes_per_exp(A, planes_bytes, valid=87.0, d=1.33):
    """Algorithmic HBM bytes of the tree kernels per expansion, SURVEY 8(d)(1):
    B_exp = sum_sel(12 A_i + 8) + 80 d + (24 + 12 A_leaf) + planes + P/v + 24 d
    (select reads P f32 / N i32 / Q f32 of each valid action at d nodes, board
    read + write per descent step, hash insert + node init, planes write, P/v
    read, backup read-modify-write).  4.77 KB for 7x7 Inflexion."""
    return d * (12.0 * valid + 8.0) + 80.0 * d + (24.0 + 12.0 * valid) + planes_bytes + (A + 1) * 4.0 + 24.0 * d


def load_pmc(G, game, impl, gemm="split"):
    """HBM-side bytes from the committed PMC passes (tools/pmc_summary.py: rocprofv3
    --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate runs, FETCH doubled per the gfx950
    correction): per split-GEMM launch, per forward of the transforms, per simulation
    step of the tree kernels.  Only valid for the workload and network form it was
    measured on (G = 4096 Inflexion 7x7, Winograd + libazg split GEMM)."""
    path = PMC_FILE_WINOGRAD.get(gemm) if impl == "winograd" else None
    if G != 4096 or game != "inflexion" or not path or not os.path.exists(path):
        return None
    d = json.load(open(path))

    def per_fwd(k):
        return (d.get(k) or {}).get("hbm_bytes_per_forward") or 0.0

    out = {"transforms": sum(per_fwd(k) for k in ("winograd_first", "winograd_mid", "winograd_out")),
           # per simulation step: select + expand / backup, fused or not (azg_sim_end_begin)
           "tree": per_fwd("select_kernel") + per_fwd("expand_backup_kernel") + per_fwd("expand_select_kernel"),
           "note": f"{os.path.relpath(path, ROOT)}: FETCH_SIZE x2 + WRITE_SIZE (split GEMM: per call; "
                   "transforms: per forward; tree: per simulation step); counts L2 misses incl. Infinity-Cache hits"}
    if per_fwd("split_gemm"):
        # per forward over the calls' launches (one per call)
        out["split_gemm_per_forward"] = per_fwd("split_gemm")
    # every kernel of a simulation step (network forward, tree, move end amortised): the games/s roofline
    out["step_total"] = sum(per_fwd(k) for k in d if not k.startswith("_"))
    return out


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=4)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--config", choices=sorted(PRESETS), default=None, help="BASELINE.json configs")
    p.add_argument("--game", choices=["inflexion", "othello"], default="inflexion")
    p.add_argument("--n", type=int, default=None)
    p.add_argument("--games", type=int, default=4096, help="concurrent games per GPU")
    p.add_argument("--sims", type=int, default=25)
    p.add_argument("--max-turns", type=int, default=343)
    p.add_argument("--evaluator", default="net", choices=["net", "stub"])
    p.add_argument("--conv", default="winograd", choices=["auto", "miopen", "azg", "winograd"],
                   help="conv2-4 implementation of the inference net (MIOpen igemm + bias/ReLU pass, libazg f32-MFMA "
                        "implicit GEMM with fused epilogue, or auto: per layer, the faster one measured at first use)")
    p.add_argument("--gemm", default="split", choices=["split", "split_blas", "f32"],
                   help="Winograd GEMMs: split-fp16 (f32-accurate, 3 fp16 MFMA products) in libazg's kernel "
                        "or hipBLASLt, or f32 MFMA")
    p.add_argument("--fc-tail", default="azg", choices=["azg", "blas"],
                   help="fc2 and [fc3 | fc4] at >= 1024 leaves: libazg split-K split GEMMs (azg) or the round-2 "
                        "hipBLASLt fp16 GEMMs (blas)")
    p.add_argument("--fc-kparts", default=None, help="with --fc-tail azg: split-K parts of fc2,fc3|fc4 (e.g. 4,2)")
    p.add_argument("--fc-small", default="on", choices=["on", "off"],
                   help="below --fc1-split-min leaves (leaves % 256 == 0): the FC tail on libazg's split GEMM, fc1 "
                        "transposed (on, nnet._fc_split_small) or the f32 hipBLASLt tail (off)")
    p.add_argument("--fc-small-kparts", default=None, help="--fc-small on: K-parts of fc1,fc2,fc3|fc4 (e.g. 18,16,8)")
    p.add_argument("--fc1-split-min", type=int, default=None,
                   help="leaves from which the FC tail runs split-fp16 on libazg (nnet.FC1_SPLIT_MIN_BATCH, 1024)")
    p.add_argument("--net", default="inference", choices=["inference", "reference"],
                   help="inference: BN-folded NHWC InferenceNet; reference: InflexionNNet as written")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-moves", type=int, default=200, help="cpu_baseline sample: first moves of one game")
    p.add_argument("--full-games", action="store_true",
                   help="time complete games (restart after warmup, play until every game ends): measured games/s")
    p.add_argument("--generation", choices=["auto", "on", "off"], default="auto",
                   help="after the timed steps, restart every game and time one whole generation (all games to "
                        "their end): measured games/s in games_per_s.  auto: on for 7x7 Inflexion at <= 25 sims "
                        "(C2, C4: ~16 s), off for the 100-200-sim configs")
    p.add_argument("--learn-iteration", choices=["auto", "on", "off"], default="auto",
                   help="after the generation pass, the rest of one Coach.learn iteration (Coach.py:102-153) on "
                        "its games: the records exchanged (all-gathered over the ranks), the example window built "
                        "on the GPU, and NNetWrapper.train_examples on it, data-parallel over the ranks; reported in "
                        "learn_iteration (self-play / exchange / train seconds, collective bytes and time per step). "
                        "auto: whenever the generation pass runs")
    p.add_argument("--train-epochs", type=int, default=10, help="--learn-iteration: epochs (NNet.py:19: 10)")
    p.add_argument("--rank0-train", type=int, default=1,
                   help="--learn-iteration with several ranks: also time the training on rank 0 alone + a weight "
                        "broadcast (train_rank0_s; 0 = skip)")
    p.add_argument("--train-window", type=int, default=200000,
                   help="--learn-iteration: examples kept from the iteration (main.py:19 maxlenOfQueue)")
    p.add_argument("--timer-every", type=int, default=25,
                   help="record the per-kernel HIP events (roofline, time split) on every N-th simulation of the "
                        "timed region only: each event record costs ~10 us of GPU idle time, which would otherwise "
                        "be charged to the throughput (1 = every simulation)")
    p.add_argument("--graph", action="store_true",
                   help="replay each move from a captured HIP graph (roofline fields then come from one extra "
                        "eager move after the timed region)")
    p.add_argument("--cpu-procs", type=int, default=0,
                   help="cpu_baseline: host cores to use (0 = the cores this process may run on, at most "
                        f"{CPU_BASELINE_MAX_CORES})")
    p.add_argument("--cpu-proc-moves", type=int, default=30,
                   help="cpu_baseline's processes x 1 thread leg: first moves of one game per process")
    # internal: collectives over gloo with ranks sharing GPUs (rehearsing --gpus N on a one-GPU box)
    p.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"], help=argparse.SUPPRESS)
    # internal: one single-threaded cpu_baseline worker (a child process, never touches the GPU)
    p.add_argument("--cpu-worker", type=int, default=None, help=argparse.SUPPRESS)
    # internal: each rank prints its rendezvous env and exits before any GPU call (tests/test_bench_cpu.py)
    p.add_argument("--print-rank-env", action="store_true", help=argparse.SUPPRESS)
    a = p.parse_args()
    if a.config:
        for k, v in PRESETS[a.config].items():
            setattr(a, k, v)
    if a.n is None:
        a.n = 7 if a.game == "inflexion" else 8
    return a


class Timer:
    """Accumulates HIP-event durations on the current stream."""

    def __init__(self):
        self.pairs = []

    def start(self):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        return e

    def stop(self, s):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        self.pairs.append((s, e))

    def total_ms(self):
        torch.cuda.synchronize()
        return sum(s.elapsed_time(e) for s, e in self.pairs)


# The GPU box gives one GPU's job 16 host cores (os.cpu_count() there shows the whole
# machine's); the CPU baseline uses at most that many.
CPU_BASELINE_MAX_CORES = 16


def host_cores():
    """Cores this process may run on (its affinity mask), and the machine's count."""
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count() or 1
    return usable, os.cpu_count() or usable


def _cpu_episode(args, depth, A, seed, max_moves, threads):
    """One oracle episode (the C restatement of the reference search) whose leaves
    are evaluated by the f32 InflexionNNet batch-1 on the CPU, like
    NNetWrapper.predict (NNet.py:78-94): (expansions, seconds, moves)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as ol
    from azg_amd.nnet import InflexionNNet
    torch.set_num_threads(threads)
    torch.manual_seed(0)
    net = InflexionNNet(n=args.n, depth=depth, action_size=A).eval()
    kind = ol.OTHELLO if args.game == "othello" else ol.INFLEXION

    def evaluator(planes):
        with torch.no_grad():
            pi, v = net(torch.from_numpy(np.array(planes, np.float32)))
        return torch.exp(pi)[0].numpy(), float(v[0, 0])

    t = time.perf_counter()
    o = ol.episode(args.n, args.max_turns, args.sims, 1, 30, seed, evaluator=evaluator, max_moves=max_moves,
                   kind=kind)
    return o["expansions"], time.perf_counter() - t, o["moves"]


def cpu_worker(args):
    """--cpu-worker SEED: one single-threaded episode sample, one JSON line on stdout."""
    from azg_amd.engine import GAMES
    _, depth, actions = GAMES[args.game]
    exp, dt, moves = _cpu_episode(args, depth, actions(args.n), args.cpu_worker, args.cpu_proc_moves, 1)
    print(json.dumps({"expansions": exp, "seconds": dt, "moves": min(moves, args.cpu_proc_moves)}), flush=True)


def cpu_baseline(args, depth, A):
    """The reference CPU path's shape on the host cores: the oracle's search with
    the same f32 network evaluated batch-1 per leaf, timed on bounded samples of
    the workload in the two arrangements BASELINE.md:20-22 measured for the
    reference itself: one process using every core as torch threads, and one
    single-threaded process per core running concurrently (the aggregate; the
    reference's best CPU arrangement, 2.2x the first).  `value` is the larger.
    The workers are child processes started with subprocess (fork + exec of a
    fresh interpreter that never touches the GPU)."""
    usable, machine = host_cores()
    cores = max(1, min(args.cpu_procs or usable, usable, CPU_BASELINE_MAX_CORES))
    exp1, dt1, moves1 = _cpu_episode(args, depth, A, 0, args.cpu_moves, cores)
    one = exp1 / dt1
    # the per-core processes: seeds 0..cores-1, the first cpu_proc_moves moves of each game
    cmd = [sys.executable, os.path.abspath(__file__), "--game", args.game, "--n", str(args.n), "--sims",
           str(args.sims), "--max-turns", str(args.max_turns), "--cpu-proc-moves", str(args.cpu_proc_moves)]
    env = dict(os.environ, OMP_NUM_THREADS="1", MKL_NUM_THREADS="1", HIP_VISIBLE_DEVICES="",
               CUDA_VISIBLE_DEVICES="", ROCR_VISIBLE_DEVICES="")
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    t = time.perf_counter()
    procs = [subprocess.Popen(cmd + ["--cpu-worker", str(i)], stdout=subprocess.PIPE, env=env, cwd=ROOT)
             for i in range(cores)]
    outs = []
    for p in procs:
        so, _ = p.communicate(timeout=600)
        if p.returncode != 0:
            raise RuntimeError(f"cpu_baseline worker exited with {p.returncode}")
        outs.append(json.loads(so.decode().strip().splitlines()[-1]))
    wall = time.perf_counter() - t
    exp_n = sum(o["expansions"] for o in outs)
    slowest = max(o["seconds"] for o in outs)
    agg = exp_n / slowest
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as ol
    kind = ol.OTHELLO if args.game == "othello" else ol.INFLEXION
    t2 = time.perf_counter()
    o2 = ol.episode(args.n, args.max_turns, args.sims, 1, 30, 0, kind=kind)
    dt2 = time.perf_counter() - t2
    best = "processes" if agg >= one else "threads"
    return {"value": max(one, agg), "unit": "node-expansions/s", "cores": cores, "kind": "port",
            "host_cpu_count": machine, "usable_cores": usable, "arrangement": best,
            "one_process_value": one,
            "one_process_sample": f"1 process x {cores} torch threads: oracle/ C MCTS + InflexionNNet f32 batch-1, "
                                  f"{args.game} {args.n}x{args.n}, seed 0, {min(moves1, args.cpu_moves)} moves x "
                                  f"{args.sims} sims = {exp1} expansions in {dt1:.1f}s",
            "processes_value": agg,
            "processes_sample": f"{cores} processes x 1 thread, concurrently: seeds 0..{cores - 1}, first "
                                f"{args.cpu_proc_moves} moves each = {exp_n} expansions; slowest process "
                                f"{slowest:.1f}s (all {wall:.1f}s wall incl. interpreter start)",
            "sample": f"max of the two arrangements ({best}); see one_process_sample / processes_sample",
            # the rate per core (the processes arrangement: one single-threaded search per
            # core) and its linear extrapolation to every core this process may use
            "per_core_value": agg / cores,
            "all_usable_cores_extrapolated_value": agg / cores * usable,
            "cores_note": (f"the GPU box grants one GPU's job a {CPU_BASELINE_MAX_CORES}-core share of the host "
                           f"(os.cpu_count() there shows the whole machine's {machine}; worker pools are to be "
                           f"sized to the share), so the baseline runs on {cores} cores; per_core_value x "
                           f"usable_cores ({usable}) is the linear extrapolation to the whole host, not a "
                           "measurement"),
            "tree_only_value": o2["expansions"] / dt2,
            "tree_only_sample": f"same search, hash evaluator, 1 thread: {o2['expansions']} expansions in {dt2:.2f}s"}


def learn_iteration(args, eng, net, rank, world, gen):
    """The rest of one Coach.learn iteration (Coach.py:102-153) after the generation pass,
    whose games are the iteration's self-play (numEps = the games per rank): the compact
    records all-gathered over the ranks (dist.gather_records, what Coach.learn's
    data-parallel mode sends), the last `train_window` examples built on the GPU
    (azg_examples, Coach.py:74-90 + the deque of :107), and NNetWrapper.train_examples on
    them (NNet.py:36-76: 10 epochs of len/512 batches, Adam), split over the ranks with one
    gradient all-reduce per step (ddp.py).  Every phase bracketed by a barrier and a
    synchronize; times are the max over ranks."""
    from azg_amd.dist import gather_records
    from azg_amd.examples import engine_examples, examples_from_records
    from azg_amd.nnet import NNetWrapper
    dev = torch.device("cuda", torch.cuda.current_device())

    def wall(t0):
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        dt = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([dt], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        return dt

    tt = eng.cfg.temp_threshold
    t0 = time.perf_counter()
    sent = 0
    if world > 1:
        rec, sent = gather_records(eng, dst=None, temp_threshold=tt)
        ex = examples_from_records(eng.game, eng.n, eng.cfg.max_turns, tt, *rec, "reference", args.train_window)
    else:
        ex = engine_examples(eng, tt, "reference", args.train_window)
    exchange_s = wall(t0)
    if args.game == "othello":
        from azg_amd.othello import OthelloGame
        game = OthelloGame(args.n)
    else:
        from azg_amd.inflexion import InflexionGame
        game = InflexionGame(args.n, max_turns=args.max_turns, max_power=6)
    w = NNetWrapper(game, {"epochs": args.train_epochs}, device=dev)
    w.nnet.load_state_dict(net.state_dict())
    # Coach.py:149's shuffle, the same permutation on every rank
    perm = torch.randperm(len(ex), generator=torch.Generator().manual_seed(0)).to(dev)
    ex = ex.index(perm)
    np.random.seed(0)
    stats = {"every": 10}
    t0 = time.perf_counter()
    w.train_examples(ex, group=dist.group.WORLD if world > 1 else None, stats=stats)
    train_s = wall(t0)
    steps = stats.get("steps", 0)
    bs = int(w.args["batch_size"])
    _, depth, _ = __import__("azg_amd.engine", fromlist=["GAMES"]).GAMES[args.game]
    flop_ex = 3 * net_flops(args.n, depth, eng.A)[0]  # forward + backward (2x) per example
    out = {"what": "one Coach.learn iteration (Coach.py:102-153): the generation pass as its self-play, then the "
                   "records exchanged, the example window built on the GPU, and NNetWrapper.train_examples",
           "ranks": world, "games": gen["games"], "selfplay_s": gen["seconds"], "exchange_examples_s": exchange_s,
           "examples": len(ex), "epochs": args.train_epochs, "batch_size": bs, "train_s": train_s,
           "train_steps": steps, "train_examples_per_s": steps * bs / train_s if train_s > 0 else None,
           "train_tflops": steps * bs * flop_ex / train_s / 1e12 if train_s > 0 else None,
           "train_flops_note": "3 x 404.3 MFLOP per example (forward + backward of InflexionNNet, SURVEY 8(a) a9)",
           "trainer": "data-parallel over the ranks (ddp.train_examples_dp)" if world > 1 else
                      "single-GPU NNetWrapper.train_examples",
           "iteration_s": gen["seconds"] + exchange_s + train_s,
           "records_sent_bytes_per_rank": sent}
    if steps and world > 1:
        out["grad_allreduce_bytes_per_step"] = stats.get("grad_allreduce_bytes", 0) / steps
        out["bn_allreduce_calls_per_step"] = stats.get("bn_allreduce_calls", 0) / steps
        out["bn_allreduce_bytes_per_step"] = stats.get("bn_allreduce_bytes", 0) / steps
        if stats.get("grad_allreduce_timed"):
            out["grad_allreduce_ms_per_step"] = stats["grad_allreduce_ms"] / stats["grad_allreduce_timed"]
            out["grad_allreduce_note"] = ("HIP events on the compute stream around the gradient all-reduce, every "
                                          f"{stats['every']}th step, rank {rank}")
    # the trainer's dominant kernel (libazg's split GEMM: the Winograd training convolutions' 9 GEMMs per
    # step -- M = V U, dV = dM U^T, dU = V^T dM for conv2-4), timed with HIP events on its stream over a
    # sample of eager steps after the timed training (a captured step records no events)
    if game.__class__.__name__ == "InflexionGame" and bs % 64 == 0:
        out["trainer_roofline"] = trainer_gemm_roofline(w, ex, dev)
    if world > 1 and args.rank0_train:
        # north_star's arrangement for comparison: the same training on rank 0 alone (the one-GPU
        # trainer: Winograd convolutions, NHWC BatchNorm, graph-replayed steps), then its weights
        # broadcast to every rank -- one collective of the state_dict instead of one all-reduce per step
        w0 = NNetWrapper(game, {"epochs": args.train_epochs}, device=dev)
        w0.nnet.load_state_dict(net.state_dict())
        np.random.seed(0)
        t0 = time.perf_counter()
        if rank == 0:
            w0.train_examples(ex)
        flat = torch.cat([t.detach().reshape(-1).float() for t in w0.nnet.state_dict().values()])
        dist.broadcast(flat, src=0)
        out["train_rank0_s"] = wall(t0)
        out["rank0_broadcast_bytes"] = flat.numel() * 4
        out["train_rank0_note"] = ("the iteration's training on rank 0 alone + one broadcast of its weights "
                                   "(north_star: examples gathered, weights broadcast), same examples and draws")
    return out


def trainer_gemm_roofline(w, ex, dev, steps=12):
    """HIP-event durations of the training step's split-GEMM launches (wino_train.GEMM_HOOK) over `steps`
    eager 512-example steps on a copy of the trained network: achieved executed-fp16 TFLOP/s against the
    dense fp16 MFMA peak, per launch on average, with the per-step GEMM share."""
    import copy
    import azg_amd.wino_train as wt
    from azg_amd.examples import ExampleSet
    w2 = copy.copy(w)
    w2.nnet = copy.deepcopy(w.nnet)
    w2.args = dict(w.args, epochs=1, train_graph=False)
    n = min(len(ex), steps * int(w2.args["batch_size"]))
    sample = ExampleSet(ex.planes[:n], ex.pis[:n], ex.vs[:n])
    pend, pairs = [], []

    def hook(what, flops):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        if what == "start":
            pend.append(e)
        else:
            pairs.append((pend.pop(), e, flops))
    state = np.random.get_state()
    wt.GEMM_HOOK = hook
    try:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        w2.train_examples(sample)
        torch.cuda.synchronize()
        step_s = (time.perf_counter() - t0) / max(n // int(w2.args["batch_size"]), 1)
    finally:
        wt.GEMM_HOOK = None
        np.random.set_state(state)
    if not pairs:
        return None
    ms = [a.elapsed_time(b) for a, b, _ in pairs]
    fl = sum(f for _, _, f in pairs)
    ach = fl / (sum(ms) / 1e3) / 1e12
    nsteps = max(n // int(w2.args["batch_size"]), 1)
    return {"bound": "mfma", "kernel": "libazg azg_split_gemm in the training step (conv2-4: M = V U, dV = dM U^T, "
                                       "dU = V^T dM; persistent 256-row and 128-row schedules)",
            "achieved": ach, "peak": F16_MFMA_PEAK_TF, "unit": "TFLOP/s", "frac": ach / F16_MFMA_PEAK_TF,
            "traffic": None, "launches": len(pairs), "avg_launch_us": sum(ms) / len(ms) * 1e3,
            "gemm_ms_per_step": sum(ms) / nsteps, "eager_step_ms": step_s * 1e3,
            "per_launch": f"{fl / len(pairs) / 1e9:.1f} GFLOP executed (3 fp16 products per f32 multiply-add) per "
                          f"launch on average over {len(pairs)} launches of {nsteps} eager steps (HIP events)"}


def rank_command(n, argv, port):
    """torchrun command for --gpus N started without a launcher: N ranks on this
    node, rendezvous on 127.0.0.1 (the driver's own form of the command)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n):
    """`bench.py --gpus N` with no WORLD_SIZE in the environment: start the N ranks
    as a child torchrun (before this process makes any GPU call; it never does) and
    exit with its status.  Rank 0 prints the JSON line."""
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(rank_command(n, sys.argv[1:], _free_port()), env=env)


def main():
    args = parse()
    if args.cpu_worker is not None:
        return cpu_worker(args)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_ranks(args.gpus)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.print_rank_env:
        print(json.dumps({"rank": rank, "local_rank": local, "world_size": world, "gpus": args.gpus,
                          "master_addr": os.environ.get("MASTER_ADDR")}), flush=True)
        return 0
    if args.dist_backend == "gloo":
        # rehearsal of the N > 1 path on fewer GPUs than ranks (tests of this script on a
        # one-GPU box): ranks share devices round-robin, collectives over gloo
        local = local % max(torch.cuda.device_count(), 1)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
        world = dist.get_world_size()
    if world != args.gpus:
        print(f"# bench: --gpus {args.gpus} but {world} rank(s) run; n_gpus reports {world}", file=sys.stderr)
    torch.cuda.set_device(local)

    import azg_amd
    from azg_amd.engine import GAMES, SelfPlayEngine
    from azg_amd.nnet import InflexionNNet, InferenceNet
    from azg_amd import dist as azg_dist

    _, depth, actions = GAMES[args.game]
    A = actions(args.n)
    flop_leaf, conv_flop_leaf = net_flops(args.n, depth, A)
    torch.manual_seed(0)
    net = InflexionNNet(n=args.n, depth=depth, action_size=A).cuda().eval()
    if args.fc_kparts:
        import azg_amd.nnet as nn_mod
        nn_mod.FC2_KPARTS, nn_mod.FC34_KPARTS = (int(x) for x in args.fc_kparts.replace("+", ",").split(","))
    if args.fc1_split_min is not None:
        import azg_amd.nnet as nn_mod
        nn_mod.FC1_SPLIT_MIN_BATCH = args.fc1_split_min
    if args.fc_small_kparts:
        import azg_amd.nnet as nn_mod
        nn_mod.FC1T_KPARTS, nn_mod.FCS_KPARTS2, nn_mod.FCS_KPARTS3 = (int(x) for x in args.fc_small_kparts.replace("+", ",").split(","))
    ev = ((InferenceNet(net, conv=args.conv, gemm=args.gemm) if args.net == "inference" else net)
          if args.evaluator == "net" else "stub")
    if args.fc_tail == "blas" and hasattr(ev, "fc_tail_azg"):
        ev.fc_tail_azg = False
    if hasattr(ev, "fc_tail_small"):
        ev.fc_tail_small = args.fc_small == "on" and hasattr(ev, "fw1_skT")
    G = args.games
    eng = SelfPlayEngine(G, sims=args.sims, cpuct=1, temp_threshold=30, max_turns=args.max_turns,
                         seed_base=0, first_game=rank * G, evaluator=ev, game=args.game, n=args.n)

    for _ in range(args.warmup):
        eng.move()
    torch.cuda.synchronize()
    st0 = eng.stats()
    t_nn, t_sel, t_exp, t_end = Timer(), Timer(), Timer(), Timer()
    t_conv = {i: Timer() for i in (2, 3, 4)}
    pending = {}
    # instrumented simulations: every args.timer_every-th one (HIP event records stall
    # the stream ~10 us each, so the others run unobserved)
    inst = {"on": False, "sims": 0, "count": 0}

    def conv_hook(i, what):
        if i not in t_conv or not inst["on"]:
            return
        if what == "start":
            pending[i] = t_conv[i].start()
        else:
            t_conv[i].stop(pending.pop(i))

    if hasattr(ev, "conv_hook"):
        ev.conv_hook = conv_hook
    # HIP events around every libazg launch of the network (split GEMM, transforms), on the
    # stream they are launched on (the current stream)
    t_kern = {"gemm": Timer(), "transform": Timer()}
    kpending = {}
    gemm_meta = []  # per timed split-GEMM launch: (layer, executed FLOPs, schedule variant)

    def kernel_hook(kind, i, what, flops=0.0, variant=None):
        if not inst["on"]:
            return
        if what == "start":
            kpending[kind] = t_kern[kind].start()
        else:
            t_kern[kind].stop(kpending.pop(kind))
            if kind == "gemm":
                gemm_meta.append((i, flops, variant))

    if hasattr(ev, "kernel_hook"):
        ev.kernel_hook = kernel_hook

    def timed_move(every=None):
        every = every or max(args.timer_every, 1)
        run = 0  # uninstrumented simulations not yet launched
        for _ in range(eng.sims):
            on = inst["count"] % every == 0
            inst["count"] += 1
            if not on:
                run += 1
                continue
            # the uninstrumented ones as the engine runs them: each expand / backup fused with
            # the next select (azg_sim_end_begin); the instrumented one split, to time its parts
            eng.simulate_many(run)
            run = 0
            inst["on"] = True
            inst["sims"] += 1
            s = t_sel.start()
            azg_amd._lib.check(eng.L.azg_sim_begin(eng.h, eng.planes.data_ptr(), eng._stream()))
            t_sel.stop(s)
            s = t_nn.start()
            P, v = eng.evaluate()
            t_nn.stop(s)
            s = t_exp.start()
            azg_amd._lib.check(eng.L.azg_sim_end(eng.h, P.data_ptr(), P.stride(0), v.data_ptr(), eng._stream()))
            t_exp.stop(s)
            inst["on"] = False
        eng.simulate_many(run)
        s = t_end.start()
        eng.move_end()
        t_end.stop(s)

    step = timed_move
    if args.graph:
        hook, khook = getattr(ev, "conv_hook", None), getattr(ev, "kernel_hook", None)
        if hook is not None:
            ev.conv_hook = None  # no event records inside the capture
        if khook is not None:
            ev.kernel_hook = None
        eng.capture_move()
        if hook is not None:
            ev.conv_hook = hook
        if khook is not None:
            ev.kernel_hook = khook
        step = eng.move
    if world > 1:
        dist.barrier()
    if args.full_games:
        eng.reset()
        torch.cuda.synchronize()
        st0 = eng.stats()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if args.full_games:
        args.steps = 0
        while eng.active() > 0:
            step()
            args.steps += 1
            if rank == 0 and args.steps % 50 == 0:
                print(f"# {args.steps} moves, {time.perf_counter() - t0:.1f}s", file=sys.stderr, flush=True)
    else:
        for _ in range(args.steps):
            step()
    sync_bytes = 0
    if world > 1:  # the per-iteration exchange of Coach.learn's data-parallel trainer: the records all-gathered
        sync_bytes = azg_dist.iteration_sync(eng, net)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    st1 = eng.stats()
    if hasattr(ev, "check_range"):
        ev.check_range()  # split GEMM operands stayed in fp16 range (raises otherwise)
    exp = st1["expansions"] - st0["expansions"]
    sims_run = st1["sims"] - st0["sims"]
    n_timed = args.steps
    if args.graph:  # kernel timings from one eager move after the timed region
        eng.drop_graph()
        if args.full_games:
            eng.reset()
        timed_move(every=1)
        n_timed = 1
    nn_ms, sel_ms, exp_ms, end_ms = t_nn.total_ms(), t_sel.total_ms(), t_exp.total_ms(), t_end.total_ms()
    if st1["error"]:
        raise RuntimeError(f"engine error {st1['error']}")

    # one whole generation after the timed steps: every game restarted and played to its end
    # (random-init games all run 344 moves), all ranks at once -- games/s measured, not estimated
    gen = None
    if not args.full_games and (args.generation == "on" or args.learn_iteration == "on"
                                or (args.generation == "auto" and args.game == "inflexion"
                                    and args.sims <= 25 and args.evaluator == "net")):
        eng.drop_graph()
        eng.reset()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        tg = time.perf_counter()
        moves = 0
        while eng.active() > 0:
            eng.move()
            moves += 1
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        gen_s = time.perf_counter() - tg
        if world > 1:
            t = torch.tensor([gen_s], dtype=torch.float64, device="cuda")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            gen_s = float(t.item())
        gen = {"games": G * world, "seconds": gen_s, "moves": moves}
        gst = eng.stats()
        if gst["error"]:
            raise RuntimeError(f"engine error {gst['error']} in the generation pass")
        gen["max_live_nodes"], gen["max_path_depth"] = gst["max_live_nodes"], gst["max_depth"]
    learn = None
    if gen is not None and args.learn_iteration != "off" and args.evaluator == "net":
        # (after the timed region: a failure here is reported in the line, not allowed to lose the
        # measured value -- every rank runs the same code, so an error raises on all of them)
        try:
            learn = learn_iteration(args, eng, net, rank, world, gen)
        except Exception as e:  # noqa: BLE001
            import traceback
            traceback.print_exc(file=sys.stderr)
            learn = {"error": f"{type(e).__name__}: {e}"[:500]}

    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        c = torch.tensor([exp, sims_run, 1], dtype=torch.float64, device="cuda")
        dist.all_reduce(c, op=dist.ReduceOp.SUM)
        exp, sims_run = int(c[0].item()), int(c[1].item())
        if int(c[2].item()) != world:  # every rank contributed its count: the ranks that ran
            raise RuntimeError(f"{int(c[2].item())} ranks reported, world size {world}")

    if rank == 0:
        value = exp / elapsed
        n_forwards = max(inst["sims"], 1)  # instrumented simulations (one forward each)
        nn_avg = nn_ms / n_forwards / 1e3
        leaves = G  # the forward is evaluated on the full [G, planes, n, n] batch
        nn_tflops = None  # set below, from the FLOPs the chosen convolution performs
        conv_ms = sum(t.total_ms() for t in t_conv.values())
        conv_avg = conv_ms / n_forwards / 1e3 if conv_ms > 0 else nn_avg
        impl = getattr(ev, "conv_impl", None) if not isinstance(ev, str) else None
        # algorithmic FLOPs of conv2-4 as computed: the Winograd path does fewer
        algo_conv_leaf = winograd_flops(args.n) if impl == "winograd" else conv_flop_leaf
        conv_flops = leaves * (algo_conv_leaf if conv_ms > 0 else flop_leaf)
        conv_tflops = conv_flops / conv_avg / 1e12 if conv_avg > 0 else 0.0
        direct_tflops = leaves * conv_flop_leaf / conv_avg / 1e12 if conv_ms > 0 and conv_avg > 0 else None
        algo_fwd_leaf = flop_leaf - conv_flop_leaf + algo_conv_leaf
        nn_tflops = leaves * algo_fwd_leaf / nn_avg / 1e12 if nn_avg > 0 else 0.0
        impls = {}
        if hasattr(ev, "_choices") or getattr(ev, "conv_impl", None):
            for i in (2, 3, 4):
                impls[i] = (next((v for (li, _), v in ev._choices.items() if li == i), "miopen")
                            if ev.conv_impl == "auto" else ev.conv_impl)
        split = impl == "winograd" and getattr(ev, "gemm", "f32") in ("split", "split_blas")

        def name(i, m):
            if m == "miopen":
                return "MIOpen igemm_fwd_gtcx35_nhwc_fp32 + libazg bias/ReLU pass"
            if m == "azg":
                return "libazg f32-MFMA implicit GEMM (LDS-DMA ring) + fused bias/ReLU"
            from azg_amd.nnet import winograd_points, winograd_seq
            g = {"split": "split-fp16 GEMMs (3 fp16 MFMA products, f32 accumulate; libazg azg_split_gemm)",
                 "split_blas": "split-fp16 GEMMs (3 fp16 MFMA products, f32 accumulate; hipBLASLt)",
                 "f32": "f32 GEMMs (hipBLASLt)"}[ev.gemm]
            sides = winograd_seq(ev.h_out[i])
            seq = "+".join(map(str, sides))
            fm = "/".join(f"F({m},3)" for m in sorted(set(sides), reverse=True))
            return (f"Winograd {seq} tiles per axis ({fm}): libazg fused transforms + "
                    f"{winograd_points(ev.h_out[i])}-point {g}")
        conv_kernel_desc = ("conv2-4 per forward: " + "; ".join(f"conv{i} {name(i, m)}" for i, m in impls.items())
                            if impls else "whole forward (no conv hook)")
        # split GEMMs execute 3 fp16 products per f32 multiply-add: priced against the fp16 MFMA peak
        mfma_mult, mfma_peak = (3, F16_MFMA_PEAK_TF) if split else (1, F32_MFMA_PEAK_TF)
        tree_s = (sel_ms + exp_ms) / 1e3
        b_exp = tree_bytes_per_exp(A, depth * args.n * args.n * 4, VALID_ACTIONS.get((args.game, args.n), 87.0))
        # expansions of the instrumented simulations (the per-simulation mean of the timed region)
        exp_inst = (exp / world) * n_forwards / max(sims_run / world / max(G, 1), 1)
        tree_gbs = exp_inst * b_exp / tree_s / 1e9 if tree_s > 0 else 0.0
        gname = f"{args.n}x{args.n} {'Inflexion' if args.game == 'inflexion' else 'Othello'}"
        out = {
            "metric": f"node-expansions/s ({gname} self-play, {args.sims} sims/move); games/s in games_per_s",
            "value": value,
            "unit": "node-expansions/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / max(args.steps, 1) * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "dtype_note": ("f32 network; Winograd GEMMs as error-compensated split-fp16 MFMA (hi*hi + lo*hi + hi*lo, "
                           "f32 accumulation; error at or below the f32 GEMM's, tests/test_gpu_nn.py)") if split else
                          "f32 network, f32 MFMA GEMMs",
            "data": f"synthetic: fresh self-play games, random-init InflexionNNet-architecture net "
                    f"(torch.manual_seed(0))" if args.evaluator == "net" else "synthetic: hash stub evaluator",
            "config": {"workload": f"{gname} self-play, {G} concurrent games/GPU x {args.sims} sims/move"
                                   + (f", max_turns {args.max_turns}" if args.game == "inflexion" else "")
                                   + f", cpuct 1, tempThreshold 30 ({args.config or 'configs[3] per GPU'})",
                       "games_per_gpu": G, "sims_per_move": args.sims, "global_games": G * world,
                       "parallelism": f"games sharded over {world} GPU(s)", "step": "one move of every game"},
            "games_per_s": (G * world / elapsed) if args.full_games else (
                gen["games"] / gen["seconds"] if gen else (
                    value / EXPANSIONS_PER_GAME_REF if args.game == "inflexion" else None)),
            "games_per_s_note": (f"measured: {G * world} complete games in {elapsed:.1f}s" if args.full_games else
                                 f"measured after the timed steps: one generation, {gen['games']} games restarted and "
                                 f"played to their end ({gen['moves']} moves) in {gen['seconds']:.1f}s over "
                                 f"{world} GPU(s)" if gen else
                                 "expansions/s / 8555 expansions per random-init game (344 moves, measured on the "
                                 "reference); bench.py --full-games or --generation on measures it"),
            "games_per_s_estimate": value / EXPANSIONS_PER_GAME_REF if args.game == "inflexion" else None,
            "expansions": exp,
            "simulations": sims_run,
            "roofline": None,  # the dominant kernel's (set below)
            "roofline_conv_span": {"bound": "mfma",
                         "kernel": conv_kernel_desc,
                         "achieved": mfma_mult * conv_tflops, "peak": mfma_peak, "unit": "TFLOP/s",
                         "frac": mfma_mult * conv_tflops / mfma_peak, "traffic": None,
                         "mfma_dtype": "fp16 (split, 3 products per f32 multiply-add)" if split else "f32",
                         "f32_equivalent_tflops": conv_tflops,
                         "direct_conv_equivalent_tflops": direct_tflops,
                         "per_launch": f"{leaves} leaves x {algo_conv_leaf / 1e6:.1f} MFLOP / {conv_avg * 1e3:.3f} ms "
                                       f"(HIP events around conv2+conv3+conv4)",
                         "forward_tflops": nn_tflops,
                         "forward_per_launch": f"{leaves} leaves x {algo_fwd_leaf / 1e6:.1f} MFLOP / "
                                               f"{nn_avg * 1e3:.3f} ms (HIP events)"},
            "roofline_tree": {"bound": "hbm", "kernel": "select_kernel + expand_backup_kernel (timed split on the instrumented simulations; the others run as the fused expand_select_kernel, whose PMC bytes per simulation step are `traffic`)",
                              "achieved": tree_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                              "frac": tree_gbs / HBM_PEAK_GBS, "traffic": None,
                              "bytes_per_expansion": b_exp,
                              "select_ms_per_sim": sel_ms / n_forwards, "expand_ms_per_sim": exp_ms / n_forwards,
                              "move_end_ms_per_move": end_ms / max(n_timed, 1)},
            "time_split": {"instrumented_sims": n_forwards, "timer_every": args.timer_every,
                           "nn_ms_per_sim": nn_ms / n_forwards, "select_ms_per_sim": sel_ms / n_forwards,
                           "expand_backup_ms_per_sim": exp_ms / n_forwards,
                           "nn_ms": nn_ms, "select_ms": sel_ms, "expand_backup_ms": exp_ms, "move_end_ms": end_ms,
                           "wall_ms": elapsed * 1e3, "graph": bool(args.graph)},
            "iteration_sync_bytes": sync_bytes,
            # the node pool's headroom (a full pool is replayed with twice the nodes by
            # Coach self-play, coach.Coach._grow); live nodes of the fullest game slot
            "tree_capacity": {"node_capacity_per_game": eng.cfg.node_capacity or 16 * args.sims + 128,
                              "max_live_nodes_timed": st1["max_live_nodes"], "max_path_depth_timed": st1["max_depth"],
                              "max_live_nodes_generation": gen["max_live_nodes"] if gen else None,
                              "max_path_depth_generation": gen["max_path_depth"] if gen else None,
                              "note": "rank 0's engine; maxima over its game slots since the last reset"},
        }
        if learn is not None:
            out["learn_iteration"] = learn
        # the dominant kernel: libazg's split GEMM (over half of the step's GPU time), its
        # launches timed with HIP events on their stream; executed MFMA FLOPs = the GEMM work
        # (Winograd: transformed points x 2 C K per leaf; fc1-fc4: the FC layers, split-K) x 3
        # fp16 products, as InferenceNet reports it per launch.  `roofline` is the kernel the
        # most GEMM time runs in -- the persistent 256-row schedule (conv2-4, fc1) -- so its
        # average launch duration is the one rocprof reports for that kernel symbol; every
        # split-GEMM launch (fc2 and [fc3 | fc4] run on the 128 / 64-row schedule) is in
        # `roofline_gemm_all`, per layer in `gemm_layers`.
        g_pairs, t_pairs = t_kern["gemm"].pairs, t_kern["transform"].pairs
        if g_pairs:
            torch.cuda.synchronize()
            durs = [st.elapsed_time(en) for st, en in g_pairs]  # ms per launch
            kname = {4: "split_gemm_persist_kernel (256 x 256 tiles, persistent)",
                     17: "split_gemm_kernel<false, 128> (128 x 256 tiles)",
                     18: "split_gemm_kernel<false, 64> (64 x 256 tiles)",
                     19: "split_gemm_384_kernel (384 x 256 tiles, persistent)"}
            lname = {2: "conv2", 3: "conv3", 4: "conv4", 5: "fc1 (split-K)", 6: "fc2 (split-K)", 7: "fc3|fc4 (split-K)"}
            by_var, by_layer = {}, {}
            for (layer, fl, var), ms in zip(gemm_meta, durs):
                by_var.setdefault(var, [0.0, 0.0, 0, set()])
                by_var[var][0] += ms
                by_var[var][1] += fl
                by_var[var][2] += 1
                by_var[var][3].add(lname.get(layer, str(layer)))
                by_layer.setdefault(layer, [0.0, 0.0, 0, var])
                by_layer[layer][0] += ms
                by_layer[layer][1] += fl
                by_layer[layer][2] += 1
            dom = max(by_var, key=lambda v: by_var[v][0])
            g_ms, g_fl, n_launch, dom_layers = by_var[dom]
            per_fwd = n_launch / n_forwards
            flops_launch = g_fl / n_launch
            ach = flops_launch / (g_ms / n_launch / 1e3) / 1e12
            all_ms, all_fl = sum(durs), sum(m[1] for m in gemm_meta)
            ach_all = all_fl / (all_ms / 1e3) / 1e12
            out["roofline"] = {
                "bound": "mfma", "kernel": f"libazg azg_split_gemm, {kname.get(dom, dom)}: "
                                           f"{', '.join(sorted(dom_layers))} (one launch per layer)",
                "achieved": ach, "peak": F16_MFMA_PEAK_TF, "unit": "TFLOP/s", "frac": ach / F16_MFMA_PEAK_TF,
                "traffic": None, "mfma_dtype": "fp16 (split, 3 products per f32 multiply-add, f32 accumulation)",
                "flops_kind": "executed fp16 MFMA FLOPs: each f32 multiply-add of the Winograd GEMMs (already 3.8x "
                              "fewer than the direct convolution's) runs as 3 fp16 products, hi.hi + lo.hi + hi.lo",
                # the same launches as f32 work (one multiply-add per product of the f32 GEMM),
                # against the f32 matrix peak -- a frac above 1 is work no f32 GEMM on this chip could do as fast
                "f32_equivalent": {"achieved": ach / 3, "peak": F32_MFMA_PEAK_TF, "unit": "TFLOP/s",
                                   "frac": ach / 3 / F32_MFMA_PEAK_TF},
                "avg_launch_us": g_ms / n_launch * 1e3, "launches": n_launch,
                "per_launch": f"{g_fl / n_forwards / 1e9:.1f} GFLOP per forward in this kernel ({leaves} leaves; 3 "
                              f"fp16 products) / {per_fwd:.0f} launches = {flops_launch / 1e9:.1f} GFLOP per launch "
                              f"(avg over the layers' shapes) / {g_ms / n_launch * 1e3:.1f} us (HIP events around "
                              "each launch)",
                "share_of_forward": all_ms / nn_ms if nn_ms > 0 else None}
            out["roofline_gemm_all"] = {
                "bound": "mfma", "kernel": "every libazg azg_split_gemm launch of the forward",
                "achieved": ach_all, "peak": F16_MFMA_PEAK_TF, "unit": "TFLOP/s", "frac": ach_all / F16_MFMA_PEAK_TF,
                "launches_per_forward": len(durs) / n_forwards}
            out["gemm_layers"] = {lname.get(k, str(k)): {"us": v[0] / v[2] * 1e3, "tflops": v[1] / (v[0] / 1e3) / 1e12,
                                                         "schedule": kname.get(v[3], v[3])}
                                  for k, v in sorted(by_layer.items())}
        if t_pairs and impl == "winograd" and getattr(ev, "gemm", "") == "split":
            tb = transform_bytes(args.n, depth, split=True)
            t_ms = t_kern["transform"].total_ms()
            gbs = leaves * tb["total"] * n_forwards / (t_ms / 1e3) / 1e9
            out["roofline_transforms"] = {
                "bound": "hbm", "kernel": "winograd_first + winograd_mid x2 + winograd_out (fused Winograd transforms)",
                "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS, "traffic": None,
                "bytes_per_leaf": tb, "us_per_forward": t_ms / n_forwards * 1e3}
        if out["roofline"] is None:  # no libazg GEMM in this configuration: the conv span is the figure
            out["roofline"] = out.pop("roofline_conv_span")
        pmc = load_pmc(G, args.game, impl, getattr(ev, "gemm", "f32"))
        if pmc:
            if "split_gemm_per_forward" in pmc and out["roofline"].get("launches"):
                out["roofline"]["traffic"] = pmc["split_gemm_per_forward"] / (out["roofline"]["launches"] / n_forwards)
            if "roofline_transforms" in out:
                out["roofline_transforms"]["traffic"] = pmc["transforms"]
            for k in ("roofline", "roofline_transforms"):
                if k in out:
                    out[k]["traffic_note"] = pmc["note"]
            out["roofline_tree"]["traffic"] = pmc["tree"]
            # north_star's "games/s as a fraction of HBM roofline": the games/s the step's measured HBM
            # bytes would allow at the 8 TB/s peak (bytes per leaf x expansions per game), against games_per_s
            if out.get("games_per_s") and args.game == "inflexion":
                per_game = pmc["step_total"] / G * EXPANSIONS_PER_GAME_REF
                peak_gps = HBM_PEAK_GBS * 1e9 / per_game * world
                out["games_roofline"] = {
                    "bound": "hbm", "achieved": out["games_per_s"], "peak": peak_gps, "unit": "games/s",
                    "frac": out["games_per_s"] / peak_gps, "bytes_per_game": per_game,
                    "note": f"PMC HBM bytes of every kernel per simulation step ({pmc['step_total'] / 1e9:.2f} GB at "
                            f"{G} leaves, {os.path.relpath(PMC_FILE_WINOGRAD['split'], ROOT)}) / {G} leaves x "
                            f"{EXPANSIONS_PER_GAME_REF} expansions per game, at {HBM_PEAK_GBS / 1e3:.0f} TB/s x "
                            f"{world} GPU(s); the step is MFMA-bound (roofline), so this is a traffic ceiling, not "
                            "the step's bound"}
        if split and getattr(ev, "gemm", "") == "split" and os.path.exists(GEMM_PMC_FILE):
            d = json.load(open(GEMM_PMC_FILE))
            out["roofline"]["mfma_busy_frac"] = d["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * d["GRBM_GUI_ACTIVE"] / 8)
            out["roofline"]["mfma_busy_note"] = (
                f"{os.path.relpath(GEMM_PMC_FILE, ROOT)}: SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 "
                "XCDs) of the split GEMM alone on conv2's shape (tools/split_gemm_pmc.py); the MFMA pipes' "
                "busy share at the clock the chip holds under this load")
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args, depth, A)
        print(json.dumps(out), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)
