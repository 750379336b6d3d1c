"""The generic plugin path with the real network on the GPU.

tests/golden/mcts_realnet_toy.json.gz: the REFERENCE Coach.executeEpisode + MCTS driven with
tests/golden/toygame.py (a plugin the engine has no kernels for) and the reference's own
NNetWrapper (its InflexionNNet sized for the game, 512 channels, torch.manual_seed(0),
batch-1 CPU f32 predict, NNet.py:78-94), 6 whole games.  Replayed by
  * the drop-in MCTS + Coach.executeEpisode with an NNetWrapper (host search, one leaf per
    GPU forward, numpy's global stream);
  * HostSelfPlay, all 6 games at once (one stream per game, each simulation step's leaves in
    one batched GPU forward);
and by Coach.learn for one iteration (host self-play -> examples -> trainer).
Counts are required equal move for move (the GPU network agrees with the CPU one to ~1e-6;
these short games meet no near-tie).
"""
import hashlib
import os
import sys

import numpy as np
import pytest
import torch

import oracle_lib as ol

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
from toygame import FourInARowGame  # noqa: E402

pytestmark = pytest.mark.gpu


class Args(dict):
    __getattr__ = dict.__getitem__

    def get(self, k, d=None):
        return dict.get(self, k, d)


def _wrapper(game):
    import azg_amd  # noqa: F401
    from azg_amd.nnet import NNetWrapper
    torch.manual_seed(0)
    return NNetWrapper(game, device="cuda")


def _check(ep, counts, actions, where):
    A = len(counts[0])
    assert len(counts) == ep["n_moves"], where
    for m, mv in enumerate(ep["moves"]):
        assert np.array_equal(counts[m], ol.golden_counts(mv, A)), f"{where} move {m}"
        assert actions[m] == mv["action"], f"{where} move {m}"


def test_dropin_real_net_generic_plugin():
    import azg_amd  # noqa: F401
    from azg_amd.coach import Coach
    from azg_amd.mcts import MCTS
    data = ol.load_json("mcts_realnet_toy.json.gz")
    cfg = data["config"]
    game = FourInARowGame(cfg["n"])
    args = Args(numMCTSSims=cfg["sims"], cpuct=cfg["cpuct"], tempThreshold=cfg["temp_threshold"])
    w = _wrapper(game)
    assert not MCTS.native(game)
    for ep in data["episodes"]:
        counts, played = [], []

        class RecMCTS(MCTS):
            def getActionProb(self, g, temp=1):
                p = super().getActionProb(g, temp)
                counts.append(self._host.root_counts(0, g))
                return p
        orig = np.random.choice

        def choice(n, p=None, _c=orig):
            a = _c(n, p=p) if p is not None else _c(n)
            if p is not None:
                played.append(int(a))
            return a
        np.random.seed(ep["seed"])
        np.random.choice = choice
        try:
            ex = Coach(game, w, args).executeEpisode((game.restarted(), RecMCTS(w, args)))
        finally:
            np.random.choice = orig
        _check(ep, counts, played, f"drop-in seed {ep['seed']}")
        pol = hashlib.sha256(np.array([e[1] for e in ex], np.float64).tobytes()).hexdigest()
        assert pol == ep["policy_sha256"] and np.random.get_state()[2] == ep["rng_pos"]


def test_batched_real_net_generic_plugin():
    import azg_amd  # noqa: F401
    from azg_amd.hostsearch import HostSelfPlay
    data = ol.load_json("mcts_realnet_toy.json.gz")
    cfg, eps = data["config"], data["episodes"]
    game = FourInARowGame(cfg["n"])
    args = Args(numMCTSSims=cfg["sims"], cpuct=cfg["cpuct"], tempThreshold=cfg["temp_threshold"])
    sp = HostSelfPlay(game, _wrapper(game), args, len(eps), first_game=eps[0]["seed"])
    res = sp.play()
    for k, (ep, (ex, rec)) in enumerate(zip(eps, res)):
        _check(ep, rec["counts"], rec["actions"], f"batched seed {ep['seed']}")
        assert rec["final"]._board.ravel().tolist() == ep["final_board"]
        assert int(sp.rng_state(k)[2]) == ep["rng_pos"]
    assert sp.search.expansions == sum(ep["expansions"] for ep in eps)


def test_learn_generic_plugin_one_iteration(tmp_path):
    """Coach.learn on a plugin without native rules: host self-play, examples, training,
    checkpoint (the arena baselines are skipped: the reference has none for it)."""
    import azg_amd  # noqa: F401
    from azg_amd.coach import Coach
    from azg_amd.nnet import NNetWrapper
    game = FourInARowGame(6)
    torch.manual_seed(0)
    w = NNetWrapper(game, dict(num_channels=32, epochs=1, batch_size=16), device="cuda")
    args = Args(numIters=1, numEps=3, tempThreshold=5, maxlenOfQueue=10**5, numMCTSSims=4, cpuct=1,
                arenaCompare=2, checkpoint=str(tmp_path), numItersForTrainExamplesHistory=5, saveExamples=True)
    c = Coach(game, w, args)
    c.learn()
    assert len(c.trainExamplesHistory) == 1 and len(c.trainExamplesHistory[0]) > 0
    assert c.last_losses.shape[1] == 2 and bool(torch.isfinite(c.last_losses).all())
    assert (tmp_path / "temp.pth.tar").exists() and (tmp_path / "checkpoint_0.pth.tar.examples").exists()
