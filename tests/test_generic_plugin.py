"""The generic plugin path (hostsearch.py) against the reference's own search.

A Game plugin the engine has no kernels for is searched on the host by calling the plugin's
methods (reference MCTS.py:62-145 over Game.py:8-181).  Pinned bit-exactly with
the hash evaluator (tests/golden/stubnet.py) against traces of the REFERENCE MCTS + Coach
driven with:
  * tests/golden/toygame.py, a third plugin (four in a row, 6 x 6, three planes, a
    two-draw random symmetry): mcts_toy.json.gz (16 games, 25 sims) and
    mcts_toy_s100.json.gz (4 games, 100 sims, cpuct 1.0, tempThreshold 4);
  * subclasses of the engine's own plugins, which the engine refuses (a subclass may
    override the rules) and the host path therefore searches: against the Othello 6x6 and
    the 40-turn Inflexion fixtures the engine itself is pinned by.
Both arrangements: the drop-in MCTS + Coach.executeEpisode on numpy's global stream (one
game, as the reference runs it), and HostSelfPlay's batched games (one stream per game,
the leaves of all games in one evaluator call).  CPU only: the stub evaluator is a plain
callable; a torch network runs on the GPU (tests/test_gpu_generic.py).
"""
import hashlib
import os
import sys

import numpy as np
import pytest

import oracle_lib as ol

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
from stubnet import stub_eval  # noqa: E402
from toygame import FourInARowGame  # noqa: E402

import azg_amd  # noqa: E402,F401
from azg_amd.coach import Coach  # noqa: E402
from azg_amd.inflexion import InflexionGame  # noqa: E402
from azg_amd.mcts import MCTS  # noqa: E402
from azg_amd.othello import OthelloGame  # noqa: E402


class Args(dict):
    __getattr__ = dict.__getitem__

    def get(self, k, d=None):
        return dict.get(self, k, d)


class HostStub:
    """The hash evaluator as a batched host callable: planes [L, C, n, n] -> (P [L, A], v [L])."""

    def __init__(self, A):
        self.A = A
        self.calls = 0
        self.leaves = 0

    def __call__(self, planes):
        self.calls += 1
        self.leaves += len(planes)
        out = [stub_eval(p, self.A) for p in planes]
        return np.stack([o[0] for o in out]), np.array([o[1][0] for o in out], np.float32)


class SubOthello(OthelloGame):
    def restarted(self):
        return SubOthello(self._n, first_mover=self._firstMover)


class SubInflexion(InflexionGame):
    def restarted(self):
        return SubInflexion(self._n, max_turns=self._max_turns, max_power=6)


SETS = {"toy": lambda c: FourInARowGame(c["n"]), "toy_s100": lambda c: FourInARowGame(c["n"]),
        "othello6": lambda c: SubOthello(c["n"]), "short": lambda c: SubInflexion(7, max_turns=c["max_turns"])}


def _fixture(name):
    d = ol.load_json(f"mcts_{name}.json.gz")
    return d["config"], d["episodes"], SETS[name](d["config"])


def _check(ep, counts, actions, examples, rng_pos, where, final=None, expansions=None):
    A = len(counts[0])
    assert len(counts) == ep["n_moves"], where
    for m, mv in enumerate(ep["moves"]):
        assert np.array_equal(counts[m], ol.golden_counts(mv, A)), f"{where} move {m}"
        assert actions[m] == mv["action"], f"{where} move {m}"
    pol = hashlib.sha256(np.array([e[1] for e in examples], np.float64).tobytes()).hexdigest()
    brd = hashlib.sha256(np.array([e[0] for e in examples], np.int64).tobytes()).hexdigest()
    assert pol == ep["policy_sha256"] and brd == ep["board_sha256"] and len(examples) == ep["n_examples"], where
    zs = [float(e[2]) for e in examples]
    rle = []
    for z in zs:
        if rle and rle[-1][0] == z:
            rle[-1][1] += 1
        else:
            rle.append([z, 1])
    assert rle == ep["z_rle"], where
    assert rng_pos == ep["rng_pos"], where
    if final is not None:
        assert final._board.astype(int).ravel().tolist() == ep["final_board"], where
        assert final.outcome.value == ep["final_outcome"], where
    if expansions is not None:
        assert expansions == ep["expansions"], where


@pytest.mark.parametrize("name", ["toy", "toy_s100", "othello6", "short"])
def test_dropin_host_search_matches_reference(name):
    """MCTS + Coach.executeEpisode over a plugin without native rules: the reference's visit
    counts, actions, examples and RNG position, game for game."""
    cfg, eps, game = _fixture(name)
    assert not MCTS.native(game)
    args = Args(numMCTSSims=cfg["sims"], cpuct=cfg["cpuct"], tempThreshold=cfg["temp_threshold"])
    for ep in eps[:6]:
        stub = HostStub(game.max_actions)
        counts, actions = [], []

        class RecMCTS(MCTS):
            def getActionProb(self, g, temp=1):
                p = super().getActionProb(g, temp)
                counts.append(self._host.root_counts(0, g))
                return p

        np.random.seed(ep["seed"])
        mcts = RecMCTS(stub, args)
        coach = Coach(game, stub, args)
        # record the actions the episode plays (not the search's descents)
        played = []
        orig_choice = np.random.choice

        def choice(n, p=None, _c=orig_choice):
            a = _c(n, p=p) if p is not None else _c(n)
            if p is not None:
                played.append(int(a))
            return a
        np.random.choice = choice
        try:
            ex = coach.executeEpisode((game.restarted(), mcts))
        finally:
            np.random.choice = orig_choice
        _check(ep, counts, played, ex, int(np.random.get_state()[2]), f"{name} seed {ep['seed']}",
               expansions=stub.leaves)
        assert mcts.stats()["expansions"] == ep["expansions"]
        assert mcts.stats()["nodes"] == ep["nodes"]


@pytest.mark.parametrize("name", ["toy", "toy_s100", "othello6", "short"])
def test_batched_host_selfplay_matches_reference(name):
    """HostSelfPlay: all of a fixture's games at once (game i seeded as the reference's
    np.random.seed(seed)), the leaves of every simulation step in one evaluator call."""
    from azg_amd.hostsearch import HostSelfPlay
    cfg, eps, game = _fixture(name)
    seeds = [ep["seed"] for ep in eps]
    assert seeds == list(range(seeds[0], seeds[0] + len(seeds)))
    args = Args(numMCTSSims=cfg["sims"], cpuct=cfg["cpuct"], tempThreshold=cfg["temp_threshold"])
    stub = HostStub(game.max_actions)
    sp = HostSelfPlay(game, stub, args, len(eps), seed_base=0, first_game=seeds[0])
    res = sp.play()
    assert stub.leaves == sum(ep["expansions"] for ep in eps)
    assert stub.calls < stub.leaves  # batched: several games' leaves per call
    for k, (ep, (ex, rec)) in enumerate(zip(eps, res)):
        # every move's root counts and action, the examples, the final board and outcome and
        # the game's own RNG position
        _check(ep, rec["counts"], rec["actions"], ex, int(sp.rng_state(k)[2]), f"{name} seed {ep['seed']}",
               final=rec["final"])


def test_coach_selfplay_batch_routes_unknown_plugins():
    """Coach.selfplay_batch on a plugin without native rules plays the host path (no engine)."""
    cfg, eps, game = _fixture("toy")
    args = Args(numMCTSSims=cfg["sims"], cpuct=cfg["cpuct"], tempThreshold=cfg["temp_threshold"])
    stub = HostStub(game.max_actions)
    c = Coach(game, stub, args)
    assert not c.native()
    ex = c.selfplay_batch(3, evaluator=stub, first_game=eps[0]["seed"])
    assert len(ex) == sum(ep["n_examples"] for ep in eps[:3])
    pol = [hashlib.sha256(np.array([e[1] for e in ex_g], np.float64).tobytes()).hexdigest()
           for ex_g in (ex[:eps[0]["n_examples"]],)]
    assert pol[0] == eps[0]["policy_sha256"]
