"""GPU parity: libazg.so (HIP) vs the reference, bit-exact on visit counts.

The search is driven by the hash evaluator (tests/golden/stubnet.py) so that
the comparison is exact: golden traces recorded from the reference
(Coach.executeEpisode + MCTS) and the C oracle must both be reproduced
count-for-count, action-for-action, expansion-for-expansion.
"""
import numpy as np
import pytest
import torch

import oracle_lib as ol

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def azg():
    import azg_amd.engine as eng
    assert torch.cuda.is_available()
    return eng


def _run(eng, seeds, cfg, **kw):
    assert list(seeds) == list(range(seeds[0], seeds[0] + len(seeds)))
    e = eng.SelfPlayEngine(len(seeds), sims=cfg["sims"], cpuct=cfg["cpuct"], temp_threshold=cfg["temp_threshold"],
                           max_turns=cfg["max_turns"], seed_base=0, first_game=seeds[0], evaluator="stub", **kw)
    e.play()
    return e, e.read_moves(), e.stats(), e.state()


def test_stub_kernel_matches_oracle(azg):
    rs = np.random.RandomState(11)
    G = 64
    planes = np.zeros((G, 4, 7, 7), np.float32)
    planes[:, 0] = rs.random_sample((G, 7, 7)) < 0.3
    planes[:, 1] = (rs.random_sample((G, 7, 7)) < 0.3) & (planes[:, 0] == 0)
    planes[:, 2] = rs.randint(0, 344, size=(G, 1, 1))
    planes[:, 3] = rs.randint(0, 2, size=(G, 1, 1))
    e = azg.SelfPlayEngine(G, evaluator="stub")
    e.planes.copy_(torch.from_numpy(planes))
    e.evaluate()
    P = e.P.cpu().numpy()
    v = e.v.cpu().numpy()
    for g in range(G):
        P2, v2 = ol.stub_eval(planes[g].astype(np.int32))
        assert np.array_equal(P[g].view(np.uint32), P2.view(np.uint32))
        assert v[g] == v2[0]


@pytest.mark.parametrize("name", ["short", "main", "pit", "sims100", "deep"])
def test_golden_traces_bit_exact(azg, name):
    data = ol.load_json(f"mcts_{name}.json.gz")
    cfg, eps = data["config"], data["episodes"]
    seeds = [ep["seed"] for ep in eps]
    cap = 16 * cfg["sims"] + 128 if cfg["sims"] < 200 else 8192
    e, rec, st, state = _run(azg, seeds, cfg, node_capacity=cap, max_depth=512)
    assert st["error"] == 0
    exp_total = 0
    for i, ep in enumerate(eps):
        assert rec["moves"][i] == ep["n_moves"], f"seed {ep['seed']}"
        for m, mv in enumerate(ep["moves"]):
            assert np.array_equal(rec["counts"][i, m], ol.golden_counts(mv)), f"seed {ep['seed']} move {m}"
            assert rec["actions"][i, m] == mv["action"], f"seed {ep['seed']} move {m}"
            assert rec["temps"][i, m] == mv["temp"]
        assert state["boards"][i].tolist() == ep["final_board"]
        assert state["players"][i] == ep["final_player"]
        assert ol.OUTCOME_VALUE[int(state["outcomes"][i])] == ep["final_outcome"]
        exp_total += ep["expansions"]
        mt, pos = e.get_rng(i)
        assert pos == ep["rng_pos"]
    assert st["expansions"] == exp_total


class Args(dict):
    __getattr__ = dict.__getitem__


@pytest.mark.parametrize("name,cap", [("deep", 0), ("short", 24), ("main", 64)])
def test_coach_recovers_a_full_node_pool(azg, name, cap):
    """Coach self-play whose node pool fills up (AZG_ERR_NODE_POOL) replays its games
    with twice the nodes per game (Coach._grow) instead of aborting the iteration, and the records
    are still the reference's, bit for bit.  `deep` (400 sims, 24 turns) at the engine's default
    capacity (16 x 400 + 128 nodes); `short` / `main` forced to 24 / 64 nodes per game, so the
    pool overflows in the first moves and is doubled until it fits."""
    from azg_amd.coach import Coach
    from azg_amd.inflexion import InflexionGame
    data = ol.load_json(f"mcts_{name}.json.gz")
    cfg, eps = data["config"], data["episodes"]
    seeds = [ep["seed"] for ep in eps]
    game = InflexionGame(7, max_turns=cfg["max_turns"], max_power=6)
    c = Coach(game, "stub", Args(numMCTSSims=cfg["sims"], cpuct=cfg["cpuct"], tempThreshold=cfg["temp_threshold"],
                                 nodeCapacity=cap))
    ex, rec = c.selfplay_batch(len(eps), first_game=seeds[0], return_records=True)
    used = c.last_capacity["node_capacity"]
    print(f"{name}: nodeCapacity {cap or 'default'} -> {used or 'default'} nodes per game")
    if cap:
        assert used >= 2 * cap
    for i, ep in enumerate(eps):
        assert rec["moves"][i] == ep["n_moves"], f"seed {ep['seed']}"
        for m, mv in enumerate(ep["moves"]):
            assert np.array_equal(rec["counts"][i, m], ol.golden_counts(mv)), f"seed {ep['seed']} move {m}"
            assert rec["actions"][i, m] == mv["action"], f"seed {ep['seed']} move {m}"
    assert len(ex) == sum(ep["n_examples"] for ep in eps)


def test_random_seeds_vs_oracle(azg):
    cfg = dict(sims=25, cpuct=1, temp_threshold=30, max_turns=60)
    seeds = list(range(1000, 1096))
    e, rec, st, state = _run(azg, seeds, cfg)
    assert st["error"] == 0
    for i, s in enumerate(seeds):
        o = ol.episode(7, cfg["max_turns"], cfg["sims"], cfg["cpuct"], cfg["temp_threshold"], s)
        m = o["moves"]
        assert rec["moves"][i] == m
        assert np.array_equal(rec["actions"][i, :m], o["actions"])
        assert np.array_equal(rec["counts"][i, :m], o["counts"])


def test_engines_on_side_streams_match_golden(azg):
    """Engines created and driven on torch side streams (non-blocking HIP streams), two
    at once, their simulations interleaved: the golden traces bit for bit.  azg_create
    zeroes its buffers on the caller's stream (a null-stream memset could land after the
    reset kernels on a non-blocking stream: every game's node pool then reads full)."""
    data = ol.load_json("mcts_short.json.gz")
    cfg, eps = data["config"], data["episodes"]
    half = len(eps) // 2
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    engs = []
    for k, s in enumerate(streams):
        with torch.cuda.stream(s):
            engs.append(azg.SelfPlayEngine(half, sims=cfg["sims"], cpuct=cfg["cpuct"],
                                           temp_threshold=cfg["temp_threshold"], max_turns=cfg["max_turns"],
                                           seed_base=0, first_game=eps[k * half]["seed"], evaluator="stub"))
    for _ in range(cfg["max_turns"] + 1):
        for _ in range(cfg["sims"]):
            for e, s in zip(engs, streams):
                with torch.cuda.stream(s):
                    e.simulate()
        for e, s in zip(engs, streams):
            with torch.cuda.stream(s):
                e.move_end()
    torch.cuda.synchronize()
    for k, e in enumerate(engs):
        assert e.stats()["error"] == 0
        rec = e.read_moves()
        for i, ep in enumerate(eps[k * half:(k + 1) * half]):
            assert rec["moves"][i] == ep["n_moves"]
            for m, mv in enumerate(ep["moves"]):
                assert np.array_equal(rec["counts"][i, m], ol.golden_counts(mv)), (ep["seed"], m)
        e.close()


@pytest.mark.parametrize("name", ["othello6", "othello8", "othello8_s200"])
def test_othello_golden_traces_bit_exact(azg, name):
    """Othello (builder-authored plugin) searched on the GPU vs the reference
    MCTS/Coach driven with the same plugin: bit-exact counts and actions."""
    data = ol.load_json(f"mcts_{name}.json.gz")
    cfg, eps = data["config"], data["episodes"]
    n, A = cfg["n"], cfg["n"] * cfg["n"] + 1
    seeds = [ep["seed"] for ep in eps]
    e = azg.SelfPlayEngine(len(seeds), sims=cfg["sims"], cpuct=cfg["cpuct"], temp_threshold=cfg["temp_threshold"],
                           game="othello", n=n, first_game=seeds[0], evaluator="stub",
                           node_capacity=16 * cfg["sims"] + 128)
    e.play()
    rec, st, state = e.read_moves(), e.stats(), e.state()
    assert st["error"] == 0
    for i, ep in enumerate(eps):
        assert rec["moves"][i] == ep["n_moves"], ep["seed"]
        for m, mv in enumerate(ep["moves"]):
            assert np.array_equal(rec["counts"][i, m], ol.golden_counts(mv, A)), (ep["seed"], m)
            assert rec["actions"][i, m] == mv["action"]
        assert state["boards"][i].tolist() == ep["final_board"]
        assert ol.OUTCOME_VALUE[int(state["outcomes"][i])] == ep["final_outcome"]
    assert st["expansions"] == sum(ep["expansions"] for ep in eps)


def test_othello_dropin_matches_reference():
    import hashlib
    import azg_amd  # noqa: F401
    from azg_amd.coach import Coach
    from azg_amd.mcts import MCTS
    from azg_amd.othello import OthelloGame

    class Args(dict):
        __getattr__ = dict.__getitem__

    data = ol.load_json("mcts_othello6.json.gz")
    cfg = data["config"]
    args = Args(numMCTSSims=cfg["sims"], cpuct=cfg["cpuct"], tempThreshold=cfg["temp_threshold"])
    for ep in data["episodes"][:4]:
        game = OthelloGame(cfg["n"])
        np.random.seed(ep["seed"])
        ex = Coach(game, "stub", args).executeEpisode((game.restarted(), MCTS("stub", args)))
        assert len(ex) == ep["n_examples"]
        pol = hashlib.sha256(np.array([e[1] for e in ex], np.float64).tobytes()).hexdigest()
        brd = hashlib.sha256(np.array([e[0] for e in ex], np.int64).tobytes()).hexdigest()
        assert pol == ep["policy_sha256"] and brd == ep["board_sha256"]


def test_engine_records_zero_copy_view(azg):
    """dist.engine_records (the tensors the RCCL example gather sends) alias the
    engine's own move records."""
    from azg_amd import dist as ad
    e = azg.SelfPlayEngine(8, sims=4, evaluator="stub", max_turns=30)
    for _ in range(3):
        e.move()
    moves, actions, counts = ad.engine_records(e)
    rec = e.read_moves()
    assert moves.device.type == "cuda" and moves.dtype == torch.int32
    assert np.array_equal(moves.cpu().numpy(), rec["moves"])
    assert np.array_equal(actions.cpu().numpy(), rec["actions"])
    assert np.array_equal(counts.cpu().numpy(), rec["counts"])


@pytest.mark.parametrize("game,n,max_turns,kind", [("inflexion", 7, 40, ol.INFLEXION), ("othello", 6, 0, ol.OTHELLO)])
def test_refill_games_match_oracle(azg, game, n, max_turns, kind):
    """Continuous batching (azg_refill): 27 games through 8 slots, each slot starting
    the next global game index as soon as its game ends; every game's record
    equals the oracle episode seeded by that index (bit-exact), whatever slot and
    moment it ran in.  Othello games differ in length, so slots refill out of step."""
    cfg = dict(sims=25, cpuct=1, temp_threshold=30)
    first, N = 700, 27
    e = azg.SelfPlayEngine(8, max_turns=max_turns if game == "inflexion" else 343, first_game=first,
                           evaluator="stub", game=game, n=n, **cfg)
    r = e.play_games(N)
    assert e.stats()["error"] == 0
    ids = r["ids"].cpu().numpy()
    assert ids.tolist() == list(range(first, first + N))
    moves, actions = r["moves"].cpu().numpy(), r["actions"].cpu().numpy()
    temps, counts = r["temps"].cpu().numpy(), r["counts"].cpu().numpy()
    lengths = set()
    for i, k in enumerate(ids):
        o = ol.episode(n, max_turns, cfg["sims"], cfg["cpuct"], cfg["temp_threshold"], int(k), kind=kind)
        m = o["moves"]
        lengths.add(m)
        assert moves[i] == m, k
        assert np.array_equal(actions[i, :m], o["actions"]), k
        assert np.array_equal(temps[i, :m], o["temps"]), k
        assert np.array_equal(counts[i, :m], o["counts"]), k
    assert e.active() == 0
    if game == "othello":
        assert len(lengths) > 1  # the slots did refill out of step


def test_no_valid_action_is_flagged_not_crashed(azg):
    """SURVEY hard part 7: a mover with no pieces and total power > 48 has no valid action
    (MCTS.py:116,131 leave best_act = -1 and the reference crashes on it).  The engine flags
    the slot with AZG_ERR_NO_ACTION and reports it (active() raises); the other slot's
    search is unaffected and bit-identical to an engine without the bad slot."""
    from azg_amd._lib import AzgError
    from azg_amd.engine import SelfPlayEngine
    cfg = dict(sims=6, cpuct=1, temp_threshold=30, max_turns=30, evaluator="stub")
    e = SelfPlayEngine(2, first_game=40, **cfg)
    board = -np.ones((7, 7), np.int8)  # 49 opponent cells of power 1: no spread, no spawn for RED
    e.set_root(0, board, turn=12, player=1)
    e.simulate()  # expands the root (all priors masked: the uniform fallback over no action)
    assert e.stats()["error"] == 0
    e.simulate()  # selects at the root: no valid action
    assert e.stats()["error"] == -5
    with pytest.raises(AzgError, match="no valid action"):
        e.active()
    for _ in range(e.sims - 2):
        e.simulate()
    ref = SelfPlayEngine(2, first_game=40, **cfg)
    for _ in range(ref.sims):
        ref.simulate()
    assert np.array_equal(e.root_counts(1), ref.root_counts(1))
    e.close()
    ref.close()
