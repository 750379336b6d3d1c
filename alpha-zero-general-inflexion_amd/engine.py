"""Batched self-play on one GPU: G concurrent games searched by libazg.so.

Replaces, for G games at once, the reference loop

    for each move:                                    Coach.executeEpisode (Coach.py:41-90)
        for numMCTSSims:  MCTS.search(game)           MCTS.py:45-46, 62-145
        pi = root visit counts ** (1/temp)            MCTS.py:48-60
        action = np.random.choice(len(pi), p=pi)      Coach.py:81
        game = game.to_next_state(action)             Coach.py:82

One *simulation step* runs one MCTS.search for every live game: the select
kernel walks each tree to a leaf and writes the leaf's randomly symmetrised
planes into a [G,4,7,7] f32 batch, the evaluator (the PyTorch-ROCm
InflexionNNet, or the hash stub used for bit-exact tests) fills P [G,343] and
v [G], and the expand/backup kernel inserts the leaves and backs the values up.
Nothing synchronises with the host inside a move.

Game slot i plays the game with global index first_game + i, seeded like
`np.random.seed(seed_base + first_game + i)`, so results do not depend on how
games are spread over GPUs.
"""
import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import check

A = 343  # InflexionGame(7) actions (the default game)
CELLS = 49

# game -> (kind code, planes per cell, actions(n))
GAMES = {"inflexion": (_lib.GAME_INFLEXION, 4, lambda n: 7 * n * n),
         "othello": (_lib.GAME_OTHELLO, 2, lambda n: n * n + 1)}


# Game plugin classes with native rules kernels (the Game.py:8-181 surface the engine
# takes its state from), matched on the exact class -- never on a name substring or
# by subclass, since a subclass may override the rules.  The reference's own
# InflexionGame (inflexion/InflexionGame.py:40) is recognised by its qualified name
# (the reference is not importable on the GPU box).  register_game() adds a plugin
# whose rules a builder has restated as kernels.
_REGISTRY = {}
_REFERENCE_CLASSES = {("inflexion.InflexionGame", "InflexionGame"): "inflexion"}
MAX_POWER_AT_SPAWN = 48  # InflexionGame.py:69 (read by the rules at :89, :95, :278)


def register_game(cls, name):
    """Map a Game plugin class to an engine game (a key of GAMES)."""
    if name not in GAMES:
        raise ValueError(f"unknown engine game {name!r}")
    _REGISTRY[cls] = name


def _registered(cls):
    if not _REGISTRY:
        from .inflexion import InflexionGame
        from .othello import OthelloGame
        register_game(InflexionGame, "inflexion")
        register_game(OthelloGame, "othello")
    name = _REGISTRY.get(cls)
    if name is None:
        name = _REFERENCE_CLASSES.get((cls.__module__, cls.__qualname__))
    return name


def game_spec(game):
    """(name, n, max_turns) of a Game plugin instance the engine has kernels for.

    Raises AzgError for any other class (an unknown plugin, or a subclass of a
    known one) and for parameters the rules kernels do not implement, instead of
    running some other game's rules.  Accepted as the reference plays them:
      * first_mover / the player to move: every quantity the engine returns is
        relative to the player to move (to_planes own/opp, the valid mask, the
        outcome, Coach.py:89's labels), and the drop-in MCTS takes the root's
        player from the instance (azg_set_root), so BLUE-first games give the
        reference's results (tests/test_gpu_dropin.py);
      * InflexionGame's max_power: stored but never read by the reference rules,
        whose power cap is the literal 6 (InflexionGame.py:66, :288), so any
        value plays those rules, here as there."""
    cls = type(game)
    name = _registered(cls)
    if name is None:
        raise _lib.AzgError(f"no native rules for Game plugin {cls.__module__}.{cls.__qualname__}: "
                            "the engine runs InflexionGame(7) and OthelloGame(6|8) "
                            "(azg_amd.engine.register_game for a plugin with its own kernels)")
    n = int(game._n)
    if name == "inflexion":
        if n != 7:
            raise _lib.AzgError(f"InflexionGame({n}): the rules kernels are built for n = 7")
        if int(getattr(game, "_max_power_at_spawn", MAX_POWER_AT_SPAWN)) != MAX_POWER_AT_SPAWN:
            raise _lib.AzgError("InflexionGame with _max_power_at_spawn != 48 has no native rules")
        max_turns = int(game._max_turns)
        if max_turns < 1:
            raise _lib.AzgError(f"InflexionGame max_turns {max_turns}: must be >= 1")
    else:
        if n not in (6, 8):
            raise _lib.AzgError(f"OthelloGame({n}): the rules kernels are built for n = 6 and 8")
        max_turns = int(getattr(game, "_max_turns", 0) or 0)
    return name, n, max_turns


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr())


class SelfPlayEngine:
    def __init__(self, num_games, *, sims=25, cpuct=1, temp_threshold=30, max_turns=343, seed_base=0,
                 first_game=0, evaluator="stub", device=None, node_capacity=0, max_depth=0, record=True,
                 gc=True, max_moves=0, game="inflexion", n=None, arena=False):
        if not torch.cuda.is_available():
            raise _lib.AzgError("SelfPlayEngine needs a HIP device (no CPU fallback)")
        if game not in GAMES:
            raise ValueError(f"unknown game {game!r}")
        kind, nplanes, actions = GAMES[game]
        n = int(n) if n is not None else (7 if game == "inflexion" else 8)
        self.game, self.n, self.A, self.cells, self.nplanes = game, n, actions(n), n * n, nplanes
        if game == "othello" and max_turns == 343:
            max_turns = 2 * n * n  # no turn limit in Othello; bounds the move records
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.G = int(num_games)
        self.sims = int(sims)
        self.evaluator = evaluator
        self.L = _lib.lib()
        with torch.cuda.device(self.device):
            self.planes = torch.zeros((self.G, nplanes, n, n), dtype=torch.float32, device=self.device)
            self.P = torch.zeros((self.G, self.A), dtype=torch.float32, device=self.device)
            self.v = torch.zeros((self.G,), dtype=torch.float32, device=self.device)
            cfg = _lib.Config(game_kind=kind, n=n, max_turns=int(max_turns), num_games=self.G,
                              sims=self.sims, temp_threshold=int(temp_threshold), cpuct=float(cpuct),
                              seed_base=int(seed_base) & 0xFFFFFFFF, pad0=0, first_game=int(first_game),
                              node_capacity=int(node_capacity), max_depth=int(max_depth),
                              max_moves=int(max_moves),
                              flags=(_lib.FLAG_GC if gc else 0) | (_lib.FLAG_RECORD if record else 0)
                              | (_lib.FLAG_ARENA if arena else 0))
            self.cfg = cfg
            h = ctypes.c_void_p()
            check(self.L.azg_create(ctypes.byref(cfg), self._stream(), ctypes.byref(h)))
            self.h = h
        self.max_moves = cfg.max_moves if cfg.max_moves > 0 else cfg.max_turns + 1
        self.record = record

    # ------------------------------------------------------------------ plumbing
    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def close(self):
        if getattr(self, "h", None):
            self.L.azg_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------ the hot path
    def evaluate(self):
        """Evaluate the current leaf batch (NNetWrapper.predict, batched).
        Returns device tensors (P [G,A] probabilities, v [G]) for sim_end."""
        ev = self.evaluator
        if isinstance(ev, str):
            if ev != "stub":
                raise ValueError(f"unknown evaluator {ev!r}")
            check(self.L.azg_stub_eval(self.h, _ptr(self.planes), _ptr(self.P), _ptr(self.v), self._stream()))
            return self.P, self.v
        with torch.no_grad():
            out_pi, out_v = ev(self.planes)
            if getattr(ev, "outputs_probs", False):
                P = out_pi
            else:  # log_softmax output: predict returns exp(pi) (NNet.py:94)
                P = torch.exp(out_pi)
            v = out_v.reshape(-1)
        if P.dtype != torch.float32 or P.stride(1) != 1 or P.shape != (self.G, self.A):
            P = P.float().contiguous()
        if v.dtype != torch.float32 or not v.is_contiguous():
            v = v.float().contiguous()
        return P, v

    def simulate(self):
        """One MCTS.search for every live game."""
        s = self._stream()
        check(self.L.azg_sim_begin(self.h, _ptr(self.planes), s))
        P, v = self.evaluate()
        check(self.L.azg_sim_end(self.h, _ptr(P), P.stride(0), _ptr(v), s))

    def simulate_many(self, k):
        """k MCTS.search calls for every live game, each backup fused with the next
        descent (azg_sim_end_begin): k + 1 tree launches instead of 2k."""
        if k <= 0:
            return
        s = self._stream()
        check(self.L.azg_sim_begin(self.h, _ptr(self.planes), s))
        for i in range(k):
            P, v = self.evaluate()
            if i + 1 < k:
                check(self.L.azg_sim_end_begin(self.h, _ptr(P), P.stride(0), _ptr(v), _ptr(self.planes), s))
            else:
                check(self.L.azg_sim_end(self.h, _ptr(P), P.stride(0), _ptr(v), s))

    def move_end(self):
        check(self.L.azg_move_end(self.h, self._stream()))

    def move(self):
        """numMCTSSims simulations + root policy / sample / apply for every live game."""
        if getattr(self, "_graph", None) is not None:
            self._graph.replay()
            return
        self.simulate_many(self.sims)
        self.move_end()

    def capture_move(self):
        """Record one whole move (select, sims x [network, expand/backup + next select] + move_end)
        as a HIP graph; later move() calls replay it (no per-kernel host launches).
        Run at least one eager move first so the network's libraries are initialised.
        Capturing launches nothing, so the games' state is unchanged."""
        g = torch.cuda.CUDAGraph()
        torch.cuda.synchronize(self.device)
        with torch.cuda.graph(g):
            self.simulate_many(self.sims)
            self.move_end()
        self._graph = g
        return g

    def drop_graph(self):
        self._graph = None

    def active(self):
        n = ctypes.c_int32()
        check(self.L.azg_active_games(self.h, ctypes.byref(n), self._stream()))
        return n.value

    # leaf batches up to this many games replay each move from a captured HIP graph in play() /
    # play_games() (graph="auto"): with few games a move's ~50 launches per simulation cost host time the
    # GPU waits for -- 64 games x 25 sims, whole games: 0.30-0.34M -> 0.39-0.40M node expansions/s; at 256
    # and 1024 the two loops measured equal (1.10-1.11M, 1.80-1.81M; profiles/r06_play_graph_ab.json)
    GRAPH_MAX_GAMES = 256

    def _auto_graph(self, graph, moved):
        """Capture the move as a HIP graph after the first eager move when graph is True, or "auto" and
        the batch is small (GRAPH_MAX_GAMES) with an InferenceNet evaluator; a refused capture keeps the
        eager loop (the same kernels: the same records)."""
        if getattr(self, "_graph", None) is not None or moved < 1:
            return
        if graph == "auto":  # (only this repo's network forms: a user's callable may run host code per call,
            from .nnet import InferenceNet  # which a replayed graph would skip)
            graph = self.G <= self.GRAPH_MAX_GAMES and isinstance(self.evaluator, InferenceNet)
        if not graph:
            return
        try:
            self.capture_move()
        except _lib.AzgError:
            raise  # an engine error is an error, not a capture limitation
        except RuntimeError as e:
            import warnings
            warnings.warn(f"SelfPlayEngine: the move could not be captured ({e}); playing eagerly")
            self._graph = None
            torch.cuda.synchronize(self.device)

    def play(self, max_moves=None, graph="auto"):
        """Play every slot's game to the end (or max_moves moves). Returns moves made."""
        m = 0
        try:
            while self.active() > 0 and (max_moves is None or m < max_moves):
                self._auto_graph(graph, m)
                self.move()
                m += 1
        finally:
            if graph == "auto":
                self.drop_graph()
        self.check_evaluator()
        return m

    def check_evaluator(self):
        """Raise FloatingPointError if the evaluator's split-fp16 GEMMs met an operand
        fp16 cannot hold since the last check (InferenceNet.check_range): its priors and
        values would be wrong, not just inexact.  play(), play_games(), the arena and the
        drop-in MCTS call this; callers rerun with nnet.replay_form."""
        chk = getattr(self.evaluator, "check_range", None)
        if chk is not None:
            chk()

    def play_games(self, num_games, first_game=None, check_every=1, graph="auto"):
        """Continuous batching (azg_refill): play the num_games games
        with global indices first_game .. first_game + num_games - 1 through the G
        slots.  A slot whose game ends hands its record off and starts the next index
        at once, so no slot waits for the longest game of a batch.  Each game is
        seeded by its own index, so its record is the one a slot of its own would
        produce (tests/test_gpu_parity.py).  Returns the records ordered by game
        index, as device tensors: {"ids" [N], "moves" [N], "actions" [N, max_moves],
        "temps" [N, max_moves], "counts" [N, max_moves, A] or None}."""
        fg = self.cfg.first_game if first_game is None else int(first_game)
        n = int(num_games)
        if n < 1:
            raise ValueError("num_games must be >= 1")
        self.reset(first_game=fg)
        dev, MM = self.device, self.max_moves
        with torch.cuda.device(dev):
            nxt = torch.tensor([fg + self.G], dtype=torch.int64, device=dev)
            cnt = torch.zeros(1, dtype=torch.int64, device=dev)
            ids = torch.full((n,), -1, dtype=torch.int64, device=dev)
            moves = torch.zeros(n, dtype=torch.int32, device=dev)
            actions = torch.zeros((n, MM), dtype=torch.int32, device=dev)
            temps = torch.zeros((n, MM), dtype=torch.int8, device=dev)
            counts = torch.zeros((n, MM, self.A), dtype=torch.int32, device=dev) if self.record else None
        args = (_ptr(nxt), fg + n, self.cfg.seed_base, _ptr(cnt), n, _ptr(ids), _ptr(moves), _ptr(actions),
                _ptr(temps), _ptr(counts) if counts is not None else None)
        k = 0
        try:
            while True:
                self._auto_graph(graph, k)
                self.move()
                check(self.L.azg_refill(self.h, *args, self._stream()))
                k += 1
                if k % check_every == 0 and self.active() == 0:
                    break
        finally:
            if graph == "auto":
                self.drop_graph()
        self.check_evaluator()
        done = int(cnt.item())
        if done != n:
            raise _lib.AzgError(f"play_games: {done} of {n} games completed")
        order = torch.argsort(ids)
        return {"ids": ids[order], "moves": moves[order], "actions": actions[order], "temps": temps[order],
                "counts": counts[order] if counts is not None else None}

    def reset(self, seed_base=None, first_game=None):
        sb = self.cfg.seed_base if seed_base is None else int(seed_base) & 0xFFFFFFFF
        fg = self.cfg.first_game if first_game is None else int(first_game)
        self.cfg.seed_base, self.cfg.first_game = sb, fg
        check(self.L.azg_reset(self.h, sb, fg, self._stream()))

    # ------------------------------------------------------------------ arena
    def set_arena(self, searcher, first_player):
        """Per slot: colour the search plays and colour to move first (+1 RED / -1 BLUE)."""
        s = np.ascontiguousarray(searcher, np.int32)
        f = np.ascontiguousarray(first_player, np.int32)
        if s.shape != (self.G,) or f.shape != (self.G,):
            raise ValueError("searcher / first_player need one entry per slot")
        check(self.L.azg_set_arena(self.h, s.ctypes.data, f.ctypes.data, self._stream()))

    def opponent_move(self, kind):
        """The baseline player's move in every slot where it is to move."""
        code = {"random": _lib.OPPONENT_RANDOM, "greedy": _lib.OPPONENT_GREEDY}[kind]
        check(self.L.azg_opponent_move(self.h, code, self._stream()))

    def follow(self, leader):
        """Play the leader engine's last move in every slot where it just moved, taking over
        the slot's numpy stream (an arena between two searchers, azg_arena_follow)."""
        check(self.L.azg_arena_follow(self.h, leader.h, self._stream()))

    # ------------------------------------------------------------------ results
    def read_moves(self, counts=True):
        G, MM = self.G, self.max_moves
        actions = np.zeros((G, MM), np.int32)
        temps = np.zeros((G, MM), np.int8)
        moves = np.zeros(G, np.int32)
        cnt = np.zeros((G, MM, self.A), np.int32) if (counts and self.record) else None
        check(self.L.azg_read_moves(self.h, actions.ctypes.data, temps.ctypes.data,
                                    cnt.ctypes.data if cnt is not None else None, moves.ctypes.data,
                                    self._stream()))
        return {"actions": actions, "temps": temps, "counts": cnt, "moves": moves}

    def state(self):
        G = self.G
        boards = np.zeros((G, self.cells), np.int8)
        turns, players, outcomes, active = (np.zeros(G, np.int32) for _ in range(4))
        check(self.L.azg_get_state(self.h, boards.ctypes.data, turns.ctypes.data, players.ctypes.data,
                                   outcomes.ctypes.data, active.ctypes.data, self._stream()))
        return {"boards": boards, "turns": turns, "players": players, "outcomes": outcomes, "active": active}

    def stats(self):
        s = np.zeros(8, np.int64)
        check(self.L.azg_stats(self.h, s.ctypes.data, self._stream()))
        return {"expansions": int(s[0]), "terminal_hits": int(s[1]), "fallbacks": int(s[2]),
                "max_depth": int(s[3]), "max_live_nodes": int(s[4]), "error": int(s[5]), "sims": int(s[6])}

    # ------------------------------------------------------------------ single-slot access (drop-in MCTS)
    def set_root(self, slot, board, turn, player):
        b = np.ascontiguousarray(np.asarray(board).reshape(-1), np.int8)
        check(self.L.azg_set_root(self.h, int(slot), b.ctypes.data, int(turn), int(player), self._stream()))

    def get_rng(self, slot):
        mt = np.zeros(624, np.uint32)
        pos = ctypes.c_int32()
        check(self.L.azg_get_rng(self.h, int(slot), mt.ctypes.data, ctypes.byref(pos), self._stream()))
        return mt, pos.value

    def set_rng(self, slot, mt, pos):
        mt = np.ascontiguousarray(mt, np.uint32)
        check(self.L.azg_set_rng(self.h, int(slot), mt.ctypes.data, int(pos), self._stream()))

    def slot_begin(self, slot, board, turn, player, mt, pos):
        """set_root + set_rng in one upload (the drop-in's per-call input)."""
        b = np.ascontiguousarray(np.asarray(board).reshape(-1), np.int8)
        mt = np.ascontiguousarray(mt, np.uint32)
        check(self.L.azg_slot_begin(self.h, int(slot), b.ctypes.data, int(turn), int(player), mt.ctypes.data,
                                    int(pos), self._stream()))

    def slot_end(self, slot):
        """root_counts + get_rng + the slot's active flag in one download; raises the slot's
        engine error.  Returns (counts [A] int32, mt [624] uint32, pos, active)."""
        c = np.zeros(self.A, np.int32)
        mt = np.zeros(624, np.uint32)
        pos, act = ctypes.c_int32(), ctypes.c_int32()
        check(self.L.azg_slot_end(self.h, int(slot), c.ctypes.data, mt.ctypes.data, ctypes.byref(pos),
                                  ctypes.byref(act), self._stream()))
        return c, mt, pos.value, act.value

    def root_counts(self, slot):
        c = np.zeros(self.A, np.int32)
        check(self.L.azg_root_counts(self.h, int(slot), c.ctypes.data, self._stream()))
        return c
