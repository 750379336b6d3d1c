"""Batched Arena: MCTSPlayer against a baseline player or another MCTSPlayer, all games at
once on the GPU.

The reference pits the trained net every pitInterval iterations (Coach.py:158-165):
Arena(MCTSPlayer(MCTS(nnet)), RandomPlayer() | GreedyPlayer(), game).playGames(
arenaCompare) runs each game in a spawn-Pool process (Arena.py:125), one
MCTS.search at a time.  Here every game is a slot of one SelfPlayEngine in
arena mode:

  * slot i < num//2 + 1 starts with RED to move, the others with BLUE
    (Arena.playGames: `(player1, player2) if i <= subtotal else (player2,
    player1)`, Arena.py:126-129); the MCTS player always plays RED
    (self.player = {RED: player1, BLUE: player2}, Arena.py:35);
  * the MCTS side searches numMCTSSims simulations with temp = 0 and plays the
    argmax of the one-hot policy (MCTSPlayer.play, InflexionPlayers.py:86-88),
    keeping its tree for the whole game (MCTSPlayer.reset per game);
  * the baseline's move is computed on the GPU (opponent_kernel): RandomPlayer
    draws np.random.choice over the valid actions from the slot's numpy stream,
    GreedyPlayer takes the best piece_count_diff after the move, ties to the
    larger action (InflexionPlayers.py:24-77);
  * results are read from RED's perspective (Arena.py:71-88).

Against a second network (`opponent` a NNetWrapper, a torch module, an evaluator or
"stub"; `opponent_args` its numMCTSSims / cpuct, default `args`) the BLUE player is
MCTSPlayer(MCTS(opponent, opponent_args)) as in Arena(player1, player2, game) with two
MCTSPlayers: a second engine holds the same games and searches for BLUE, and after each
side's move the other engine plays the same action in its copy and takes over the slot's
numpy stream (azg_arena_follow), so both players draw from one stream per game as the
reference's do in its one process.  Each player keeps its own tree for the whole game.

Each slot has its own numpy stream seeded by its game index (the reference's
Pool workers draw from unseeded per-process streams, so its arena results are
not reproducible run to run).
"""
import logging

import numpy as np

from .engine import SelfPlayEngine, game_spec
from .flags import GameOutcome

log = logging.getLogger(__name__)

_OUT = {0: GameOutcome.ONGOING, 1: GameOutcome.DRAW, 2: GameOutcome.WON, 3: GameOutcome.LOST}


class BatchedArena:
    def __init__(self, game, nnet, args, opponent="random", evaluator=None, seed_base=0, first_game=0,
                 opponent_args=None, opponent_evaluator=None):
        self.game, self.nnet, self.args, self.opponent = game, nnet, args, opponent
        self.searching_opponent = not (isinstance(opponent, str) and opponent in ("random", "greedy"))
        if isinstance(opponent, str) and opponent != "stub" and self.searching_opponent:
            raise ValueError(f"unknown opponent {opponent!r}")
        if evaluator is None:
            evaluator = self._inference_form(nnet, "split")
        self.evaluator = evaluator
        self.opponent_args = opponent_args if opponent_args is not None else args
        self.opponent_evaluator = None
        if self.searching_opponent:
            self.opponent_evaluator = (opponent_evaluator if opponent_evaluator is not None
                                       else self._inference_form(opponent, "split"))
        self.seed_base, self.first_game = seed_base, first_game
        self.last_engine_state = None

    @staticmethod
    def _inference_form(nnet, gemm):
        from .nnet import InferenceNet, NNetWrapper, replay_form
        if not isinstance(nnet, NNetWrapper):
            return nnet
        return replay_form(nnet.nnet) if gemm == "f32" else InferenceNet(nnet.nnet, gemm=gemm)

    def playGames(self, num, verbose=False):
        """Arena.playGames (Arena.py:90-142): (MCTS player wins, baseline wins, draws).
        If the split-fp16 network met an operand out of fp16 range, the games are
        replayed (same seeds, same result as a first run) with nnet.replay_form."""
        if not (isinstance(num, int) and num >= 2):
            raise AssertionError("num must be an int >= 2")
        try:
            return self._play(num)
        except FloatingPointError:
            f32 = self._inference_form(self.nnet, "f32")
            f32_opp = self._inference_form(self.opponent, "f32") if self.searching_opponent else None
            if f32 is self.evaluator and f32_opp is self.opponent_evaluator:
                raise
            log.warning("arena: split-fp16 operand out of range; replaying with the f32 replay form")
            self.evaluator, self.opponent_evaluator = f32, f32_opp
            return self._play(num)

    def _engine(self, num, args, evaluator):
        name, n, max_turns = game_spec(self.game)
        return SelfPlayEngine(num, sims=int(args.numMCTSSims), cpuct=args.cpuct, temp_threshold=0,
                              max_turns=max_turns, game=name, n=n, seed_base=self.seed_base,
                              first_game=self.first_game, evaluator=evaluator, record=False, arena=True)

    def _play(self, num):
        subtotal = num // 2
        first = np.where(np.arange(num) <= subtotal, 1, -1).astype(np.int32)
        eng = self._engine(num, self.args, self.evaluator)
        engs = [eng]
        try:
            eng.set_arena(np.ones(num, np.int32), first)
            if self.searching_opponent:
                blue = self._engine(num, self.opponent_args, self.opponent_evaluator)
                engs.append(blue)
                blue.set_arena(-np.ones(num, np.int32), first)
            while eng.active() > 0:
                eng.move()  # searches in the slots where the MCTS player (RED) is to move
                if self.searching_opponent:
                    blue.follow(eng)
                    blue.move()  # BLUE's MCTS player, in its own engine and trees
                    eng.follow(blue)
                    blue.active()  # raises on an error in the BLUE engine's slots
                else:
                    eng.opponent_move(self.opponent)
            for e in engs:
                e.check_evaluator()
            st = eng.state()
            self.last_moves = eng.read_moves(counts=False)
            if self.searching_opponent:  # the BLUE engine's copy of the same games
                self.last_opponent_moves = blue.read_moves(counts=False)
            err = next((x for x in (e.stats()["error"] for e in engs) if x), 0)
        finally:
            for e in engs:
                e.close()
        if err:
            raise RuntimeError(f"arena engine error {err}")
        self.last_engine_state = st
        one = two = draws = 0
        for g in range(num):
            out = _OUT[int(st["outcomes"][g])]
            if int(st["players"][g]) != 1:  # game.player = RED: the setter flips the outcome
                out = out.opposite()
            if out == GameOutcome.WON:
                one += 1
            elif out == GameOutcome.LOST:
                two += 1
            elif out == GameOutcome.DRAW:
                draws += 1
            else:
                raise ValueError(f"Unexpected game status: {out}")
        return one, two, draws
