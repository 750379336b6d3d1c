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
import pickle
import random
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

    def _engine(self, num_games, evaluator, seed_base, first_game):
        from .engine import SelfPlayEngine, game_spec
        name, n, max_turns = game_spec(self.game)
        return SelfPlayEngine(num_games, sims=int(self.args.numMCTSSims), cpuct=self.args.cpuct,
                              temp_threshold=int(self.args.tempThreshold), max_turns=max_turns, game=name, n=n,
                              seed_base=seed_base, first_game=first_game,
                              evaluator=evaluator if evaluator is not None else self.evaluator())

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
        """run(evaluator) -> result; if the split-fp16 network met an operand out of
        fp16 range (FloatingPointError from SelfPlayEngine.check_evaluator), rerun
        with nnet.replay_form.  Games are seeded by their index, so the rerun's
        records are the ones a first f32 run would have produced."""
        ev = evaluator if evaluator is not None else self.evaluator()
        try:
            return run(ev)
        except FloatingPointError:
            if evaluator is not None or ev is self.nnet:
                raise
            log.warning("self-play: split-fp16 operand out of range; replaying with the f32 replay form")
            return run(self.evaluator(gemm="f32"))

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

        def run(ev):
            eng = self._engine(num_games, ev, seed_base, first_game)
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
            def run(ev):
                eng = self._engine(slots, ev, seed_base, first_game)
                try:
                    return eng.play_games(num_games, first_game=first_game)
                finally:
                    eng.close()
            r = self._range_checked(run, evaluator)
            name, n, max_turns = game_spec(self.game)
            return examples_from_records(name, n, max_turns, int(self.args.tempThreshold), r["moves"],
                                         r["actions"], r["counts"], self.label_mode, maxlen)

        def run(ev):
            eng = self._engine(num_games, ev, seed_base, first_game)
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

        def run(ev):
            eng = self._engine(eps, ev, 0, first)
            try:
                eng.play()
            except BaseException:
                eng.close()
                raise
            return eng
        # The ranks agree on how self-play went before any of them enters the record
        # exchange (flag: 0 ok, 1 a split-fp16 operand out of fp16 range, 2 any other
        # error).  On 1 EVERY rank replays its games with nnet.replay_form, together: no
        # rank waits in the gather while another replays (which could outlast the process
        # group's timeout), and the iteration's records are those of an all-f32 run
        # whatever the sharding.  On 2 every rank raises, instead of the healthy ranks
        # blocking in the gather until the timeout.
        ev = self.evaluator()
        eng, flag_v, err = None, 0, None
        try:
            eng = run(ev)
        except FloatingPointError as e:
            flag_v, err = (2, e) if ev is self.nnet else (1, None)
        except Exception as e:  # noqa: BLE001 -- reported to every rank, re-raised below
            flag_v, err = 2, e
        dev = (torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl"
               else torch.device("cpu"))
        flag = torch.tensor([flag_v], dtype=torch.int64, device=dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
        flag_v = int(flag.item())
        if flag_v == 2:
            if eng is not None:
                eng.close()
            if err is not None:
                raise err
            raise RuntimeError("self-play failed on another rank; this rank stops with it")
        if flag_v == 1:
            log.warning("self-play: split-fp16 operand out of range on a rank; all ranks replay with "
                        "the f32 replay form")
            if eng is not None:
                eng.close()
            eng = run(self.evaluator(gemm="f32"))
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
        from .examples import ExampleSet
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
            perm = list(range(len(train)))
            if trainer:
                random.shuffle(perm)  # shuffle(trainExamples), Coach.py:149
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
        """Coach.py:170-176: the history as a pickled list of deques of
        (board, pi, z) tuples in checkpoint_{iteration}.pth.tar.examples."""
        folder = self.args.checkpoint
        os.makedirs(folder, exist_ok=True)
        filename = os.path.join(folder, self.getCheckpointFile(iteration) + ".examples")
        hist = [deque(h.to_list() if hasattr(h, "to_list") else h, maxlen=int(self.args.maxlenOfQueue))
                for h in self.trainExamplesHistory]
        with open(filename, "wb+") as f:
            pickle.Pickler(f).dump(hist)

    def loadTrainExamples(self, device=None):
        """Coach.py:178-193 for a file this Coach (or the reference) wrote: the
        history comes back as device ExampleSets; self-play of iteration 1 is
        skipped.  A missing file raises FileNotFoundError (the reference asks on
        stdin)."""
        from .examples import ExampleSet
        model_file = os.path.join(self.args.load_folder_file[0], self.args.load_folder_file[1])
        examples_file = model_file + ".examples"
        if not os.path.isfile(examples_file):
            raise FileNotFoundError(f'File "{examples_file}" with trainExamples not found')
        with open(examples_file, "rb") as f:
            hist = pickle.Unpickler(f).load()
        dev = device or self.nnet.device
        self.trainExamplesHistory = [ExampleSet.from_list(list(h), dev) for h in hist if len(h)]
        self.skipFirstSelfPlay = True


def examples_from_record(template, actions, temps, counts, moves, label_mode="reference"):
    """Rebuild one game's examples by replaying its recorded actions."""
    g = template.restarted()
    planes, pis, players = [], [], []
    for m in range(moves):
        c = counts[m].astype(np.int64)
        if temps[m]:
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
