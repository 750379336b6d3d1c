"""Search parity with the PRODUCTION evaluator: the engine driven by the real
network reproduces the reference's visit counts with the reference's own network.

Fixtures (tests/golden/make_golden.py `realnet`): the reference Coach.executeEpisode
(Coach.py:41-90) + MCTS (MCTS.py:33-145) with the reference NNetWrapper
(inflexion/pytorch/NNet.py:78-94, batch-1 CPU f32) over the 512-channel
InflexionNNet built under torch.manual_seed(0) -- whole 344-move episodes at
main.py's 25 sims, and 40-turn games at C3's 100 sims.

Each is replayed three ways, all of which must give the reference's visit counts
on EVERY move (the north_star's "bit-exact on visit counts for a fixed RNG seed"),
actions and RNG position:
  * the drop-in MCTS + Coach.executeEpisode with an NNetWrapper (batch-1 forward of
    the reference module on the GPU);
  * SelfPlayEngine with InferenceNet(gemm="split") at 4096 concurrent games -- the
    benchmarked path (Winograd transforms, split-fp16 MFMA GEMMs, split-K fc1);
  * the same with InferenceNet(gemm="f32") (f32 hipBLASLt GEMMs).
pi returned by getActionProb is a function of the counts (MCTS.py:48-60), so equal
counts give pi exactly (tolerance 0, inside the north_star's 1e-5).

If a near-tie flips, the failure names the seed, the move, and the root's prior
margin: the largest |P_engine - P_reference| at that root against the smallest
gap between two valid actions' priors.
"""
import numpy as np
import pytest
import torch

import oracle_lib as ol

pytestmark = pytest.mark.gpu

G_ENGINE = 4096  # the benchmarked leaf batch (split-K fc1 needs >= 1024 leaves)


class Args(dict):
    __getattr__ = dict.__getitem__


def _ref_net():
    import azg_amd  # noqa: F401
    from azg_amd.nnet import InflexionNNet
    torch.manual_seed(0)
    return InflexionNNet().cuda().eval()


def _margin_report(net, evaluator, board, turn, player, max_turns):
    """Root priors at a failing move: the evaluator on the GPU (at the batch size
    it ran at) against the reference's arithmetic (the module on the CPU, batch 1)."""
    import copy
    from azg_amd.flags import PlayerColour
    from azg_amd.inflexion import InflexionGame
    g = InflexionGame(7, max_turns=max_turns, board=np.asarray(board).reshape(7, 7).astype(int), curr_turn=turn,
                      curr_player=PlayerColour.RED if player == 1 else PlayerColour.BLUE)
    x = torch.as_tensor(g.to_planes(), dtype=torch.float32).unsqueeze(0)
    with torch.no_grad():
        p_ref = torch.exp(copy.deepcopy(net).cpu()(x)[0][0]).numpy()
        if isinstance(evaluator, str) or evaluator is None:  # the drop-in: the module, batch 1
            p_ev = torch.exp(net(x.cuda())[0][0]).cpu().numpy()
        else:
            xb = x.cuda().expand(G_ENGINE, *x.shape[1:]).contiguous()
            p_ev = evaluator(xb)[0][0].cpu().numpy()
    valid = g.valid_actions_mask().astype(bool)
    pv = np.sort(p_ref[valid])
    gap = float(np.min(np.diff(pv))) if len(pv) > 1 else float("inf")
    return f"root prior error {float(np.max(np.abs(p_ev - p_ref)[valid])):.3g}, smallest prior gap {gap:.3g}"


def _check_episode(ep, counts, actions, n_moves, where, report):
    for m, mv in enumerate(ep["moves"]):
        want = ol.golden_counts(mv)
        if m >= n_moves or not np.array_equal(counts[m], want) or actions[m] != mv["action"]:
            got = counts[m] if m < n_moves else None
            diff = np.nonzero(got != want)[0].tolist() if got is not None else []
            raise AssertionError(f"{where}: seed {ep['seed']} move {m} (turn {mv['turn']}): counts differ at "
                                 f"actions {diff[:8]} (engine {got[diff[:8]].tolist() if got is not None else None}, "
                                 f"reference {want[diff[:8]].tolist()}); {report(mv)}")
    assert n_moves == ep["n_moves"], (where, ep["seed"])


@pytest.mark.parametrize("name,k", [("realnet_main", 0), ("realnet_main", 1), ("realnet_sims100", 0)])
def test_dropin_mcts_real_net(name, k):
    """Drop-in MCTS + Coach.executeEpisode with an NNetWrapper, whole episodes."""
    import hashlib
    import azg_amd  # noqa: F401
    from azg_amd.coach import Coach
    from azg_amd.inflexion import InflexionGame
    from azg_amd.mcts import MCTS
    from azg_amd.nnet import NNetWrapper

    data = ol.load_json(f"mcts_{name}.json.gz")
    cfg, ep = data["config"], data["episodes"][k]
    args = Args(numMCTSSims=cfg["sims"], cpuct=cfg["cpuct"], tempThreshold=cfg["temp_threshold"])
    game = InflexionGame(7, max_turns=cfg["max_turns"], max_power=6)
    torch.manual_seed(0)
    wrapper = NNetWrapper(game, device="cuda")
    counts, actions = [], []

    class RecMCTS(MCTS):
        def getActionProb(self, g, temp=1):
            p = super().getActionProb(g, temp)
            counts.append(self._engine.root_counts(0))
            return p

    orig = InflexionGame.to_next_state

    def tns(self, a):
        actions.append(int(a))
        return orig(self, a)
    np.random.seed(ep["seed"])
    InflexionGame.to_next_state = tns
    try:
        ex = Coach(game, wrapper, args).executeEpisode((game.restarted(), RecMCTS(wrapper, args)))
    finally:
        InflexionGame.to_next_state = orig
    net = wrapper.nnet.eval()
    _check_episode(ep, counts, actions, len(counts), "drop-in MCTS",
                   lambda mv: _margin_report(net, None, mv["board"], mv["turn"], 1 - 2 * (mv["turn"] % 2),
                                             cfg["max_turns"]))
    pol = hashlib.sha256(np.array([e[1] for e in ex], np.float64).tobytes()).hexdigest()
    assert pol == ep["policy_sha256"] and len(ex) == ep["n_examples"]
    assert np.random.get_state()[2] == ep["rng_pos"]


@pytest.mark.parametrize("gemm", ["split", "f32"])
@pytest.mark.parametrize("name", ["realnet_main", "realnet_sims100"])
def test_engine_real_net_4096_games(name, gemm):
    """The batched engine with the production evaluator at 4096 games: the
    fixture's seeds are game slots of a full-size run (seed = slot index +
    first_game), the other slots are ordinary games in the same leaf batches."""
    import azg_amd  # noqa: F401
    from azg_amd.engine import SelfPlayEngine
    from azg_amd.nnet import InferenceNet

    data = ol.load_json(f"mcts_{name}.json.gz")
    cfg, eps = data["config"], data["episodes"]
    seeds = [ep["seed"] for ep in eps]
    assert seeds == list(range(seeds[0], seeds[0] + len(seeds)))
    net = _ref_net()
    ev = InferenceNet(net, gemm=gemm)
    e = SelfPlayEngine(G_ENGINE, sims=cfg["sims"], cpuct=cfg["cpuct"], temp_threshold=cfg["temp_threshold"],
                       max_turns=cfg["max_turns"], seed_base=0, first_game=seeds[0], evaluator=ev)
    e.play()
    st = e.stats()
    assert st["error"] == 0
    rec = e.read_moves()
    state = e.state()
    for i, ep in enumerate(eps):
        _check_episode(ep, rec["counts"][i], rec["actions"][i], int(rec["moves"][i]), f"engine gemm={gemm}",
                       lambda mv: _margin_report(net, ev, mv["board"], mv["turn"], 1 - 2 * (mv["turn"] % 2),
                                                 cfg["max_turns"]))
        assert state["boards"][i].tolist() == ep["final_board"]
        assert ol.OUTCOME_VALUE[int(state["outcomes"][i])] == ep["final_outcome"]
        assert e.get_rng(i)[1] == ep["rng_pos"]
    e.close()
