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
the engine's move records.
"""
import numpy as np

from .flags import GameOutcome, PlayerColour
from .inflexion import InflexionGame

N_SYM = 36


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
        if not (game._curr_turn == 0 and game.outcome == GameOutcome.ONGOING):
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
            if game.outcome != GameOutcome.ONGOING:
                return build_examples(game, planes, pis, players, game, self.label_mode)

    def selfplay_batch(self, num_games, evaluator=None, seed_base=0, first_game=0, return_records=False):
        """Play num_games complete games concurrently on the GPU engine and
        return their examples (same format as executeEpisode)."""
        from .engine import SelfPlayEngine, game_spec
        g0 = self.game
        name, n, max_turns = game_spec(g0)
        eng = SelfPlayEngine(num_games, sims=int(self.args.numMCTSSims), cpuct=self.args.cpuct,
                             temp_threshold=int(self.args.tempThreshold), max_turns=max_turns, game=name, n=n,
                             seed_base=seed_base, first_game=first_game,
                             evaluator=evaluator if evaluator is not None else self.nnet)
        try:
            eng.play()
            rec = eng.read_moves()
        finally:
            eng.close()
        examples = []
        for i in range(num_games):
            examples += examples_from_record(g0, rec["actions"][i], rec["temps"][i], rec["counts"][i],
                                             int(rec["moves"][i]), self.label_mode)
        return (examples, rec) if return_records else examples


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
