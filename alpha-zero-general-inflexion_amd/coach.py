"""Self-play episodes with the reference Coach's interface and example format.

`Coach.executeEpisode((game, mcts))` restates Coach.py:41-90 over the drop-in
GPU MCTS: per move temp = int(step < tempThreshold), pi from
mcts.getActionProb, 36 symmetric copies of the pi plane and of the planes,
action = np.random.choice(len(pi), p=pi), step; returns
[(planes int64[4,n,n], pi list, z)].

`label_mode` selects how z is assigned:
  "reference" (default) reproduces Coach.py:79 exactly, where the player list
      grows by the *cumulative* number of examples each move (SURVEY.md
      finding 6: about half the labels are wrong), so outputs are identical to
      the reference's;
  "per_move" labels each example with the player of its own move.

`selfplay_batch` plays many games at once on the batched engine (per-game
numpy streams seeded by global game index) and builds the same examples from
the engine's move records on the host; `selfplay_examples` builds them on the
GPU (examples.py) and `learn` runs the reference's iteration loop
(Coach.py:92-165) with self-play, examples and training all on the device.
"""
import logging
import os
from collections import deque

import numpy as np
import torch

from .flags import PlayerColour, ongoing
from .inflexion import InflexionGame

N_SYM = 36
log = logging.getLogger(__name__)


def _label_players(move_players, label_mode, n_sym=N_SYM):
    """Player attached to each of the n_sym*L examples (Coach.py:77-79)."""
    L = len(move_players)
    idx = np.arange(n_sym * L)
    if label_mode == "per_move":
        block = idx // n_sym
    elif label_mode == "reference":
        # after move m (1-based) the list holds n_sym * m * (m + 1) / 2 entries
        cum = n_sym * np.arange(1, L + 1) * np.arange(2, L + 2) // 2
        block = np.searchsorted(cum, idx, side="right")
    else:
        raise ValueError(f"unknown label_mode {label_mode!r}")
    return np.asarray(move_players)[block]


def build_examples(game, move_planes, move_pis, move_players, final, label_mode="reference"):
    boards, policies = [], []
    for planes, pi in zip(move_planes, move_pis):
        policies += game.symmetries(np.asarray(pi).reshape(game.policy_shape))
        boards += game.symmetries(planes)
    n_sym = len(boards) // max(len(move_planes), 1)
    players = _label_players(move_players, label_mode, n_sym)
    v = final.outcome.value
    return [(b, p.ravel().tolist(), v if pl == final.player.num else -v)
            for b, p, pl in zip(boards, policies, players)]


class Coach:
    def __init__(self, game, nnet, args, label_mode="reference"):
        self.game = game
        self.nnet = nnet
        self.args = args
        self.label_mode = label_mode
        self.trainExamplesHistory = []
        self.skipFirstSelfPlay = False

    def executeEpisode(self, args):
        game, mcts = args
        if not (game._curr_turn == 0 and ongoing(game.outcome)):
            raise AssertionError("executeEpisode needs a fresh game")
        planes, pis, players = [], [], []
        step = 0
        while True:
            step += 1
            temp = int(step < self.args.tempThreshold)
            pi = mcts.getActionProb(game, temp=temp)
            planes.append(game.to_planes())
            pis.append(pi)
            players.append(game.player.num)
            action = np.random.choice(len(pi), p=pi)
            game = game.to_next_state(action)
            if not ongoing(game.outcome):
                return build_examples(game, planes, pis, players, game, self.label_mode)

    def _engine(self, num_games, evaluator, seed_base, first_game, node_capacity=0, max_depth=0):
        from .engine import SelfPlayEngine, game_spec
        name, n, max_turns = game_spec(self.game)
        return SelfPlayEngine(num_games, sims=int(self.args.numMCTSSims), cpuct=self.args.cpuct,
                              temp_threshold=int(self.args.tempThreshold), max_turns=max_turns, game=name, n=n,
                              seed_base=seed_base, first_game=first_game,
                              evaluator=evaluator if evaluator is not None else self.evaluator(),
                              node_capacity=node_capacity, max_depth=max_depth)

    def _capacity(self):
        """The engine's per-game tree capacity for self-play: args.nodeCapacity / args.maxDepth
        (0 or absent: the engine's defaults, 16 numMCTSSims + 128 nodes and a 256-node path)."""
        get = self.args.get if hasattr(self.args, "get") else (lambda k, d=None: d)
        return {"node_capacity": int(get("nodeCapacity", 0) or 0), "max_depth": int(get("maxDepth", 0) or 0)}

    def _grow(self, cap, code):
        """The capacity after a run that filled it: a full node pool (AZG_ERR_NODE_POOL) doubles the
        nodes per game, a path deeper than max_depth (AZG_ERR_PATH) doubles the path.  Games are
        seeded by their index and the tree's contents do not depend on the capacity (nodes are
        found by key; GC frees by turn), so the rerun's records are those a large-enough first
        run gives."""
        from ._lib import ERR_NODE_POOL, ERR_PATH, AzgError
        cap = dict(cap)
        if code == ERR_NODE_POOL:
            cur = cap["node_capacity"] or 16 * int(self.args.numMCTSSims) + 128
            if 2 * cur >= 1 << 21:
                raise AzgError(f"self-play: node pool full at {cur} nodes per game (the engine's limit is 2^21)",
                               code)
            cap["node_capacity"] = 2 * cur
            log.warning("self-play: a game's node pool filled up; replaying with %d nodes per game", 2 * cur)
        elif code == ERR_PATH:
            cur = cap["max_depth"] or 256
            if 2 * cur > 1 << 16:
                raise AzgError(f"self-play: search path deeper than {cur}", code)
            cap["max_depth"] = 2 * cur
            log.warning("self-play: a search path outgrew max_depth; replaying with max_depth %d", 2 * cur)
        else:
            raise ValueError(code)
        self.last_capacity = cap
        return cap

    def evaluator(self, gemm="split"):
        """The leaf evaluator for the engine: an NNetWrapper's current weights as
        the inference form (BN folded, NHWC; nnet.InferenceNet), else self.nnet
        itself (a module, or "stub").  gemm="f32" gives the out-of-fp16-range
        fallback, nnet.replay_form (direct f32 convolutions)."""
        from .nnet import InferenceNet, NNetWrapper, replay_form
        if isinstance(self.nnet, NNetWrapper):
            return replay_form(self.nnet.nnet) if gemm == "f32" else InferenceNet(self.nnet.nnet, gemm=gemm)
        return self.nnet

    def _range_checked(self, run, evaluator):
        """run(evaluator, **capacity) -> result, rerun until it fits: if the split-fp16 network
        met an operand out of fp16 range (FloatingPointError from SelfPlayEngine.check_evaluator),
        with nnet.replay_form; if a game's tree outgrew the engine's node pool or path
        (AzgError AZG_ERR_NODE_POOL / AZG_ERR_PATH), with twice that capacity (_grow).  Games are
        seeded by their index, so the rerun's records are the ones a first run with that
        evaluator and capacity would have produced."""
        from ._lib import ERR_NODE_POOL, ERR_PATH, AzgError
        ev = evaluator if evaluator is not None else self.evaluator()
        cap = self._capacity()
        self.last_capacity = cap
        while True:
            try:
                return run(ev, **cap)
            except FloatingPointError:
                if evaluator is not None or ev is self.nnet or getattr(ev, "gemm", None) == "f32":
                    raise
                log.warning("self-play: split-fp16 operand out of range; replaying with the f32 replay form")
                ev = self.evaluator(gemm="f32")
            except AzgError as e:
                if e.code not in (ERR_NODE_POOL, ERR_PATH):
                    raise
                cap = self._grow(cap, e.code)

    def native(self):
        """Whether the engine has rules kernels for self.game (else the generic host path)."""
        from .mcts import MCTS
        return MCTS.native(self.game)

    def _host_selfplay(self, num_games, seed_base, first_game, evaluator=None):
        """The generic plugin path (hostsearch.HostSelfPlay): num_games episodes of a plugin
        without native rules, searched on the host with the leaves batched to the GPU network;
        returns [(examples, record)] per game."""
        from .hostsearch import HostSelfPlay
        sp = HostSelfPlay(self.game, evaluator if evaluator is not None else self.nnet, self.args, num_games,
                          seed_base, first_game)
        return sp.play(self.label_mode)

    def selfplay_batch(self, num_games, evaluator=None, seed_base=0, first_game=0, return_records=False):
        """Play num_games complete games concurrently on the GPU engine and
        return their examples (same format as executeEpisode).  A plugin without
        native rules plays on the generic host path (hostsearch.py)."""
        g0 = self.game
        if not self.native():
            res = self._host_selfplay(num_games, seed_base, first_game, evaluator)
            examples = [e for ex, _ in res for e in ex]
            return (examples, [r for _, r in res]) if return_records else examples

        def run(ev, **cap):
            eng = self._engine(num_games, ev, seed_base, first_game, **cap)
            try:
                eng.play()
                return eng.read_moves()
            finally:
                eng.close()
        rec = self._range_checked(run, evaluator)
        examples = []
        for i in range(num_games):
            examples += examples_from_record(g0, rec["actions"][i], rec["temps"][i], rec["counts"][i],
                                             int(rec["moves"][i]), self.label_mode)
        return (examples, rec) if return_records else examples

    # ---------------------------------------------------------------- learn loop
    def selfplay_examples(self, num_games, evaluator=None, seed_base=0, first_game=0, maxlen=None):
        """One iteration's self-play (Coach.py:106-112) as num_games concurrent
        games (or, with args.selfplaySlots = S < num_games, through S engine slots
        that refill as games end); the examples (last maxlen, default
        args.maxlenOfQueue) are built on the GPU and returned as a device ExampleSet."""
        from .engine import game_spec
        from .examples import ExampleSet, engine_examples, examples_from_records
        maxlen = int(self.args.maxlenOfQueue if maxlen is None else maxlen)
        if not self.native():
            ex = [e for exs, _ in self._host_selfplay(num_games, seed_base, first_game, evaluator) for e in exs]
            return ExampleSet.from_list(ex[-maxlen:], self.nnet.device)
        slots = int(self.args.get("selfplaySlots", 0) or 0)
        if 0 < slots < num_games:
            # continuous batching: num_games games through `slots` engine slots
            # (azg_refill); same examples, game for game, as one slot per game
            def run(ev, **cap):
                eng = self._engine(slots, ev, seed_base, first_game, **cap)
                try:
                    return eng.play_games(num_games, first_game=first_game)
                finally:
                    eng.close()
            r = self._range_checked(run, evaluator)
            name, n, max_turns = game_spec(self.game)
            return examples_from_records(name, n, max_turns, int(self.args.tempThreshold), r["moves"],
                                         r["actions"], r["counts"], self.label_mode, maxlen)

        def run(ev, **cap):
            eng = self._engine(num_games, ev, seed_base, first_game, **cap)
            try:
                eng.play()
                return engine_examples(eng, int(self.args.tempThreshold), self.label_mode, maxlen)
            finally:
                eng.close()
        return self._range_checked(run, evaluator)

    def _dp_train(self):
        """Multi-rank training mode: "ddp" (default: every rank builds the iteration's
        examples from all-gathered records and trains its slice of every batch,
        ddp.train_examples_dp) or "rank0" (rank 0 alone trains on gathered records and
        broadcasts its weights; the round-3 arrangement)."""
        mode = (self.args.get("distributedTrain", "ddp") if hasattr(self.args, "get") else "ddp") or "ddp"
        if mode not in ("ddp", "rank0"):
            raise ValueError(f"distributedTrain must be 'ddp' or 'rank0', got {mode!r}")
        return mode == "ddp"

    def _selfplay_iteration(self, i, group, all_ranks=False):
        """Self-play of iteration i over all ranks; examples land on the trainer (rank 0),
        or on every rank with all_ranks (data-parallel training)."""
        import torch.distributed as dist
        from .dist import broadcast_weights, gather_records
        from .engine import game_spec
        from .examples import examples_from_records
        eps = int(self.args.numEps)
        if group is None and not (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1):
            return self.selfplay_examples(eps, first_game=(i - 1) * eps)
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        if not all_ranks:  # data-parallel training keeps the ranks' weights equal by construction
            broadcast_weights(self.nnet.nnet, src=0, group=group)
        first = ((i - 1) * world + rank) * eps
        if not self.native():
            return self._host_selfplay_iteration(first, eps, group, all_ranks)

        def run(ev, **cap):
            eng = self._engine(eps, ev, 0, first, **cap)
            try:
                eng.play()
            except BaseException:
                eng.close()
                raise
            return eng
        # The ranks agree on how self-play went before any of them enters the record
        # exchange: flags [fp16, pool, path, error] MAX-reduced (a split-fp16 operand out of
        # fp16 range; a game's tree outgrew the node pool / the search path, AZG_ERR_NODE_POOL /
        # AZG_ERR_PATH; anything else).  On fp16 or capacity EVERY rank
        # replays its games -- with nnet.replay_form and / or twice the capacity -- together:
        # no rank waits in the gather while another replays (which could outlast the process
        # group's timeout), and the iteration's records are those of a first run with that
        # evaluator and capacity whatever the sharding.  On an error every rank raises,
        # instead of the healthy ranks blocking in the gather until the timeout.
        from ._lib import ERR_NODE_POOL, ERR_PATH, AzgError
        ev = self.evaluator()
        cap = self._capacity()
        dev = (torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl"
               else torch.device("cpu"))
        replayed_f32 = False
        while True:
            eng, flags, err = None, [0, 0, 0, 0], None
            try:
                eng = run(ev, **cap)
            except FloatingPointError as e:
                if ev is self.nnet or replayed_f32:
                    flags[3], err = 1, e
                else:
                    flags[0] = 1
            except AzgError as e:
                if e.code == ERR_NODE_POOL:
                    flags[1] = 1
                elif e.code == ERR_PATH:
                    flags[2] = 1
                else:
                    flags[3], err = 1, e
            except Exception as e:  # noqa: BLE001 -- reported to every rank, re-raised below
                flags[3], err = 1, e
            flag = torch.tensor(flags, dtype=torch.int64, device=dev)
            dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
            f16, pool, path, bad = (int(x) for x in flag.tolist())
            if not (f16 or pool or path or bad):
                break
            if eng is not None:
                eng.close()
            if bad:
                if err is not None:
                    raise err
                raise RuntimeError("self-play failed on another rank; this rank stops with it")
            if f16:
                log.warning("self-play: split-fp16 operand out of range on a rank; all ranks replay with "
                            "the f32 replay form")
                ev, replayed_f32 = self.evaluator(gemm="f32"), True
            if pool:
                cap = self._grow(cap, ERR_NODE_POOL)
            if path:
                cap = self._grow(cap, ERR_PATH)
        flag_v = int(replayed_f32)
        self.last_replayed_f32 = flag_v == 1
        try:
            rec, self.last_sent_bytes = gather_records(eng, dst=None if all_ranks else 0, group=group,
                                                       temp_threshold=int(self.args.tempThreshold))
        finally:
            eng.close()
        if rec is None:
            return None
        name, n, max_turns = game_spec(self.game)
        mv, act, cnt = rec
        return examples_from_records(name, n, max_turns, int(self.args.tempThreshold), mv, act, cnt,
                                     self.label_mode, int(self.args.maxlenOfQueue))

    def _host_selfplay_iteration(self, first, eps, group, all_ranks):
        """A multi-rank iteration of a plugin without native rules: each rank plays its games
        on the host path and the example lists travel as objects (all ranks with all_ranks,
        else the trainer)."""
        import torch.distributed as dist
        from .examples import ExampleSet
        # the ranks agree on how self-play went before the object exchange, as the native path
        # does: a rank that raised would otherwise leave the others blocked in the
        # gather until the process group's timeout
        ex, err = None, None
        try:
            ex = [e for exs, _ in self._host_selfplay(eps, 0, first) for e in exs]
        except Exception as e:  # noqa: BLE001 -- reported to every rank, re-raised below
            err = e
        dev = (torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl"
               else torch.device("cpu"))
        flag = torch.tensor([0 if err is None else 2], dtype=torch.int64, device=dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
        if int(flag.item()):
            if err is not None:
                raise err
            raise RuntimeError("host self-play failed on another rank; this rank stops with it")
        world = dist.get_world_size(group)
        if all_ranks:
            parts = [None] * world
            dist.all_gather_object(parts, ex, group=group)
        else:
            parts = [None] * world if dist.get_rank(group) == 0 else None
            from .dist import group_src
            dist.gather_object(ex, parts, dst=group_src(group, 0), group=group)
            if parts is None:
                return None
        allex = [e for p in parts for e in p]
        return ExampleSet.from_list(allex[-int(self.args.maxlenOfQueue):], self.nnet.device)

    def learn(self, group=None, pit=True):
        """Coach.learn (Coach.py:92-165): per iteration, numEps self-play games
        (on every rank when torch.distributed is initialised: the engine plays
        numEps games per rank), the example history window, the examples file,
        training (NNetWrapper.train_examples), temp.pth.tar and, every pitInterval
        iterations, the arena against the baselines.

        With several ranks and args.distributedTrain "ddp" (the default) every rank
        receives all ranks' records (all-gather), builds the same examples and history,
        and trains data-parallel (ddp.train_examples_dp: the reference's batches split
        over the ranks, one gradient all-reduce per step), so all GPUs train and the
        weights need no broadcast; "rank0" gathers the records to rank 0, which trains
        alone and broadcasts its weights at the start of the next iteration."""
        import torch.distributed as dist
        from .examples import ExampleSet, shuffle_perm
        distributed = group is not None or (dist.is_available() and dist.is_initialized()
                                            and dist.get_world_size() > 1)
        trainer = not distributed or dist.get_rank(group) == 0
        ddp = distributed and self._dp_train()
        dp_group = (group if group is not None else dist.group.WORLD) if ddp else None
        if distributed:
            self.agree_skip_first(group)
        if ddp:
            from .dist import broadcast_weights
            from .ddp import broadcast_example_sets
            broadcast_weights(self.nnet.nnet, src=0, group=group)  # one start for every rank
            if self.skipFirstSelfPlay:  # loadTrainExamples ran on the trainer only
                dev = self.nnet.device if dist.get_backend(group) == "nccl" else torch.device("cpu")
                hist = broadcast_example_sets(self.trainExamplesHistory if trainer else None, 0, group, dev)
                self.trainExamplesHistory = [ExampleSet(h.planes.to(self.nnet.device), h.pis.to(self.nnet.device),
                                                        h.vs.to(self.nnet.device)) for h in hist]
        pit_interval = 5
        for i in range(1, int(self.args.numIters) + 1):
            log.info("Starting Iter #%d ...", i)
            if not self.skipFirstSelfPlay or i > 1:
                ex = self._selfplay_iteration(i, group, all_ranks=ddp)
                if trainer or ddp:
                    self.trainExamplesHistory.append(ex)
            if not (trainer or ddp):
                continue
            if len(self.trainExamplesHistory) > int(self.args.numItersForTrainExamplesHistory):
                log.warning("Removing the oldest entry in trainExamples. len(trainExamplesHistory) = %d",
                            len(self.trainExamplesHistory))
                self.trainExamplesHistory.pop(0)
            if trainer and self.args.get("saveExamples", True):
                self.saveTrainExamples(i - 1)
            train = ExampleSet.cat(self.trainExamplesHistory)
            perm = np.arange(len(train), dtype=np.int64)
            if trainer:
                # shuffle(trainExamples), Coach.py:149: random.shuffle's permutation and stream
                # position, drawn natively (examples.shuffle_perm; 4M examples: ~2.2 s in Python)
                perm = shuffle_perm(len(train))
            if ddp:  # the trainer's shuffle on every rank
                from .ddp import broadcast_perm
                dev = self.nnet.device if dist.get_backend(group) == "nccl" else torch.device("cpu")
                perm = broadcast_perm(perm, 0, group, dev)
            self.last_losses = self.nnet.train_examples(
                train.index(torch.as_tensor(perm, dtype=torch.long, device=train.vs.device)), group=dp_group)
            if trainer:
                self.nnet.save_checkpoint(folder=self.args.checkpoint, filename="temp.pth.tar")
                if pit and i % pit_interval == 0:
                    self.pit_baselines()
        if distributed and not ddp:
            from .dist import broadcast_weights
            broadcast_weights(self.nnet.nnet, src=0, group=group)

    def agree_skip_first(self, group=None):
        """Make every rank follow the trainer's skipFirstSelfPlay (loadTrainExamples is
        naturally called on the trainer only), so all ranks enter iteration 1's
        collectives alike."""
        import torch.distributed as dist
        from .dist import group_src
        dev = (torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl"
               else torch.device("cpu"))
        flag = torch.tensor([int(self.skipFirstSelfPlay)], dtype=torch.int64, device=dev)
        dist.broadcast(flag, src=group_src(group, 0), group=group)
        self.skipFirstSelfPlay = bool(flag.item())
        return self.skipFirstSelfPlay

    def pit_baselines(self):
        """Coach.py:158-165: the new net's MCTSPlayer against RandomPlayer and
        GreedyPlayer, args.arenaCompare games each (batched on the GPU)."""
        from .arena import BatchedArena
        res = {}
        if not self.native():  # the baselines (InflexionPlayers.py) exist for the engine's games only
            log.warning("pit_baselines: no Random/Greedy baseline players for %s; skipped", type(self.game).__name__)
            self.last_pit = res
            return res
        for opp in ("random", "greedy"):
            arena = BatchedArena(self.game, self.nnet, self.args, opponent=opp)
            p1, p2, draws = arena.playGames(int(self.args.arenaCompare))
            log.info("NEW/%s WINS : %d / %d ; DRAWS : %d", opp, p1, p2, draws)
            res[opp] = (p1, p2, draws)
        self.last_pit = res
        return res

    # ---------------------------------------------------------------- example files
    def getCheckpointFile(self, iteration):
        return "checkpoint_" + str(iteration) + ".pth.tar"

    def saveTrainExamples(self, iteration):
        """Coach.py:170-176: the history in checkpoint_{iteration}.pth.tar.examples.

        args.examplesFormat "azg" (default): a JSON manifest naming one array file per window,
        each window written once, when it is first saved (examples.write_manifest): a save
        costs O(the iteration's new window) instead of re-pickling every window's Python
        tuples (the reference's 20 x 200,000-example history is ~1.4e9 Python floats per
        save).  "reference": the reference's own pickle of a list of deques of (board, pi, z)
        tuples, streamed (examples.export_reference_examples), for a reference Coach to load.
        loadTrainExamples reads both."""
        from .examples import export_reference_examples, write_manifest
        folder = self.args.checkpoint
        os.makedirs(folder, exist_ok=True)
        filename = os.path.join(folder, self.getCheckpointFile(iteration) + ".examples")
        fmt = self.args.get("examplesFormat", "azg") if hasattr(self.args, "get") else "azg"
        hist = [h if not isinstance(h, (list, deque)) else _as_example_set(h, self.nnet.device)
                for h in self.trainExamplesHistory]
        if fmt == "reference":
            export_reference_examples(hist, filename, int(self.args.maxlenOfQueue))
        elif fmt == "azg":
            self.last_windows_written = write_manifest(hist, filename, int(self.args.maxlenOfQueue), iteration)
        else:
            raise ValueError(f"examplesFormat must be 'azg' or 'reference', got {fmt!r}")

    def export_reference_examples(self, filename):
        """Write the current history as the reference's examples pickle (Coach.py:170-176)."""
        from .examples import export_reference_examples
        export_reference_examples([_as_example_set(h, self.nnet.device) for h in self.trainExamplesHistory],
                                  filename, int(self.args.maxlenOfQueue))

    def loadTrainExamples(self, device=None):
        """Coach.py:178-193 for a file this Coach (either format) or the reference wrote: the
        history comes back as device ExampleSets; self-play of iteration 1 is skipped.  A
        missing file raises FileNotFoundError (the reference asks on stdin)."""
        from .examples import read_examples_file
        model_file = os.path.join(self.args.load_folder_file[0], self.args.load_folder_file[1])
        examples_file = model_file + ".examples"
        if not os.path.isfile(examples_file):
            raise FileNotFoundError(f'File "{examples_file}" with trainExamples not found')
        self.trainExamplesHistory = read_examples_file(examples_file, device or self.nnet.device)
        self.skipFirstSelfPlay = True


def _as_example_set(h, device):
    from .examples import ExampleSet
    return h if isinstance(h, ExampleSet) else ExampleSet.from_list(list(h), device)


def examples_from_record(template, actions, temps, counts, moves, label_mode="reference"):
    """Rebuild one game's examples by replaying its recorded actions."""
    g = template.restarted()
    planes, pis, players = [], [], []
    for m in range(moves):
        if temps[m]:  # (only temperature-1 moves read their counts: rank-gathered records hold just those rows)
            c = counts[m].astype(np.int64)
            pi = c / c.sum()
        else:
            pi = np.zeros(len(c), dtype=np.int8)
            pi[actions[m]] = 1
        planes.append(g.to_planes())
        pis.append(pi)
        players.append(g.player.num)
        g = g.to_next_state(int(actions[m]))
    return build_examples(g, planes, pis, players, g, label_mode)


__all__ = ["Coach", "build_examples", "examples_from_record", "InflexionGame", "PlayerColour"]
