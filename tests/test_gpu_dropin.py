"""Drop-in interface parity on the GPU: azg_amd's MCTS + Coach reproduce the
reference Coach.executeEpisode exactly (visit counts, actions, examples)."""
import hashlib

import numpy as np
import pytest
import torch

import oracle_lib as ol

pytestmark = pytest.mark.gpu


class Args(dict):
    __getattr__ = dict.__getitem__


def _episode(seed, cfg, label_mode="reference"):
    import azg_amd  # noqa: F401
    from azg_amd.coach import Coach
    from azg_amd.inflexion import InflexionGame
    from azg_amd.mcts import MCTS

    args = Args(numMCTSSims=cfg["sims"], cpuct=cfg["cpuct"], tempThreshold=cfg["temp_threshold"])
    game = InflexionGame(7, max_turns=cfg["max_turns"], max_power=6)
    counts = []

    class RecMCTS(MCTS):
        def getActionProb(self, g, temp=1):
            p = super().getActionProb(g, temp)
            counts.append(self._engine.root_counts(0))
            return p

    coach = Coach(game, "stub", args, label_mode=label_mode)
    np.random.seed(seed)
    ex = coach.executeEpisode((game.restarted(), RecMCTS("stub", args)))
    return ex, counts


@pytest.mark.parametrize("name,limit", [("short", 16), ("main", 2), ("pit", 1)])
def test_execute_episode_matches_reference(name, limit):
    data = ol.load_json(f"mcts_{name}.json.gz")
    cfg = data["config"]
    for ep in data["episodes"][:limit]:
        ex, counts = _episode(ep["seed"], cfg)
        assert len(counts) == ep["n_moves"]
        for m, mv in enumerate(ep["moves"]):
            assert np.array_equal(counts[m], ol.golden_counts(mv)), (ep["seed"], m)
        assert len(ex) == ep["n_examples"]
        zs = [float(e[2]) for e in ex]
        rle = []
        for z in zs:
            if rle and rle[-1][0] == z:
                rle[-1][1] += 1
            else:
                rle.append([z, 1])
        assert rle == ep["z_rle"]
        pol = hashlib.sha256(np.array([e[1] for e in ex], np.float64).tobytes()).hexdigest()
        brd = hashlib.sha256(np.array([e[0] for e in ex], np.int64).tobytes()).hexdigest()
        assert pol == ep["policy_sha256"] and brd == ep["board_sha256"]
        st = np.random.get_state()
        assert st[2] == ep["rng_pos"]
        assert np.random.randint(0, 2**32, size=4, dtype=np.uint32).tolist() == ep["rng_next"]


def test_batched_selfplay_examples_match_reference():
    import azg_amd  # noqa: F401
    from azg_amd.coach import Coach
    from azg_amd.inflexion import InflexionGame

    data = ol.load_json("mcts_short.json.gz")
    cfg, eps = data["config"], data["episodes"]
    args = Args(numMCTSSims=cfg["sims"], cpuct=cfg["cpuct"], tempThreshold=cfg["temp_threshold"])
    game = InflexionGame(7, max_turns=cfg["max_turns"], max_power=6)
    coach = Coach(game, "stub", args)
    ex, rec = coach.selfplay_batch(len(eps), evaluator="stub", first_game=eps[0]["seed"], return_records=True)
    off = 0
    for i, ep in enumerate(eps):
        n = ep["n_examples"]
        mine = ex[off:off + n]
        off += n
        pol = hashlib.sha256(np.array([e[1] for e in mine], np.float64).tobytes()).hexdigest()
        brd = hashlib.sha256(np.array([e[0] for e in mine], np.int64).tobytes()).hexdigest()
        assert pol == ep["policy_sha256"] and brd == ep["board_sha256"], ep["seed"]
    assert off == len(ex)


def test_real_net_dropin_runs_and_is_close_to_cpu_net():
    """The real InflexionNNet through the drop-in: GPU f32 leaf values vs the CPU
    network on the same planes (tolerance 1e-5 relative, north_star)."""
    import azg_amd  # noqa: F401
    from azg_amd.nnet import NNetWrapper
    d = dict(np.load(ol.os.path.join(ol.GOLDEN, "nnet_golden.npz")))
    torch.manual_seed(0)
    w = NNetWrapper(device="cuda")
    for planes, P, v in zip(d["planes"][:16], d["P"][:16], d["v"][:16]):
        p2, v2 = w.predict(planes.astype(np.int64))
        np.testing.assert_allclose(p2, P, rtol=1e-5, atol=1e-7)
        np.testing.assert_allclose(v2[0], v, rtol=1e-5, atol=1e-6)
