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


def test_dropin_pool_sized_for_whole_game_and_full_pool_raises():
    """the drop-in's node pool holds a whole game's tree (sims per move x
    moves), and a search that still fills a (deliberately small) pool raises instead of
    returning counts from a truncated search."""
    import azg_amd  # noqa: F401
    from azg_amd._lib import AzgError
    from azg_amd.inflexion import InflexionGame
    from azg_amd.mcts import MCTS, whole_game_capacity

    args = Args(numMCTSSims=25, cpuct=1, tempThreshold=30)
    game = InflexionGame(7, max_turns=343, max_power=6)
    assert whole_game_capacity(25, game) == 25 * 344 + 64
    assert whole_game_capacity(100, game) == 100 * 344 + 64
    np.random.seed(3)
    small = MCTS("stub", args, node_capacity=40)
    g = game.restarted()
    small.getActionProb(g, temp=1)  # 25 nodes: fits
    g = g.to_next_state(int(np.argmax(small._engine.root_counts(0))))
    with pytest.raises(AzgError):
        small.getActionProb(g, temp=1)  # up to 50 nodes: the pool of 40 fills
    np.random.seed(3)
    full = MCTS("stub", args)
    assert full._engine_for(game).cfg.node_capacity == whole_game_capacity(25, game)


def test_engine_raises_on_split_gemm_range_flag():
    """a split-fp16 evaluator whose range flag trips makes play() raise, and the
    Coach replays the games with the f32-GEMM form (same records as an f32 run)."""
    import azg_amd  # noqa: F401
    from azg_amd.coach import Coach
    from azg_amd.engine import SelfPlayEngine
    from azg_amd.inflexion import InflexionGame
    from azg_amd.nnet import InferenceNet, InflexionNNet, NNetWrapper

    torch.manual_seed(0)
    net = InflexionNNet().cuda().eval()
    fast = InferenceNet(net)
    eng = SelfPlayEngine(4, evaluator=fast, sims=2, max_turns=6)
    fast.overflow.fill_(1)  # as the GEMM's range check would
    with pytest.raises(FloatingPointError):
        eng.play()
    eng.close()
    assert int(fast.overflow.item()) == 0  # the check clears the sticky flag

    args = Args(numMCTSSims=2, cpuct=1, tempThreshold=3, maxlenOfQueue=200000)
    game = InflexionGame(7, max_turns=6, max_power=6)
    wrapper = NNetWrapper(game)
    wrapper.nnet = net
    coach = Coach(game, wrapper, args)
    made = []

    def evaluator(gemm="split"):
        ev = InferenceNet(net, gemm=gemm)
        if gemm == "split":
            ev.overflow.fill_(1)
        made.append(gemm)
        return ev
    coach.evaluator = evaluator
    ex = coach.selfplay_examples(4)
    assert made == ["split", "f32"]
    coach.evaluator = lambda gemm="split": InferenceNet(net, gemm="f32")
    ref = coach.selfplay_examples(4)
    assert torch.equal(ex.pis, ref.pis) and torch.equal(ex.planes, ref.planes) and torch.equal(ex.vs, ref.vs)


def _overflowing_net():
    """A network whose conv2 activations exceed fp16's range (|v| > 65504) while its
    outputs stay ordinary: bn2's scale x1e5 and bn3's / 1e5 (BN folds into the convs,
    InflexionNNet.py:39-45), the kind of large-activation net a trained one can be."""
    import azg_amd  # noqa: F401
    from azg_amd.nnet import InflexionNNet
    torch.manual_seed(0)
    net = InflexionNNet().cuda().eval()
    with torch.no_grad():
        net.bn2.weight.mul_(1e5)
        net.bn3.weight.div_(1e5)
    return net


def test_replay_form_accurate_where_split_overflows():
    """the out-of-range fallback (nnet.replay_form: direct f32 convolutions)
    holds the 1e-5 tolerance against the reference module on exactly the networks that
    trip the split form's range flag."""
    from azg_amd.engine import SelfPlayEngine
    from azg_amd.nnet import InferenceNet, replay_form
    net = _overflowing_net()
    e = SelfPlayEngine(1024, evaluator="stub", sims=3, max_turns=343)
    e.move()
    e.move()
    e.simulate()
    x = e.planes.clone()  # a real 1024-leaf batch
    e.close()
    split = InferenceNet(net)
    with torch.no_grad():
        split(x)
    with pytest.raises(FloatingPointError):
        split.check_range()
    rf = replay_form(net)
    with torch.no_grad():
        p, v = rf(x)
        logp, v_ref = net(x)
    torch.testing.assert_close(p, torch.exp(logp), rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(v.reshape(-1), v_ref.reshape(-1), rtol=1e-5, atol=1e-6)
    assert float(v_ref.abs().max()) < 0.999  # outputs not saturated: the comparison means something
    rf.check_range()  # the f32 form has no range flag to trip


def test_blue_first_dropin_matches_red_first_reference():
    """A BLUE-first InflexionGame (Game.py:14-24 first_mover) through the drop-in:
    everything the search sees is relative to the player to move, so its visit
    counts and examples are the reference's RED-first ones (mcts_short fixture) with
    the board's signs flipped."""
    import azg_amd  # noqa: F401
    from azg_amd.coach import Coach
    from azg_amd.flags import PlayerColour
    from azg_amd.inflexion import InflexionGame
    from azg_amd.mcts import MCTS

    data = ol.load_json("mcts_short.json.gz")
    cfg = data["config"]
    args = Args(numMCTSSims=cfg["sims"], cpuct=cfg["cpuct"], tempThreshold=cfg["temp_threshold"])
    game = InflexionGame(7, first_mover=PlayerColour.BLUE, max_turns=cfg["max_turns"], max_power=6)
    for ep in data["episodes"][:3]:
        counts = []

        class RecMCTS(MCTS):
            def getActionProb(self, g, temp=1):
                p = super().getActionProb(g, temp)
                counts.append(self._engine.root_counts(0))
                return p
        np.random.seed(ep["seed"])
        ex = Coach(game, "stub", args).executeEpisode((game.restarted(), RecMCTS("stub", args)))
        assert len(counts) == ep["n_moves"]
        for m, mv in enumerate(ep["moves"]):
            assert np.array_equal(counts[m], ol.golden_counts(mv)), (ep["seed"], m)
        pol = hashlib.sha256(np.array([e[1] for e in ex], np.float64).tobytes()).hexdigest()
        brd = hashlib.sha256(np.array([e[0] for e in ex], np.int64).tobytes()).hexdigest()
        assert pol == ep["policy_sha256"] and brd == ep["board_sha256"] and len(ex) == ep["n_examples"]


@pytest.mark.parametrize("game_name", ["inflexion", "othello6"])
def test_dropin_graph_replay_matches_eager(game_name):
    """The drop-in replays each call's numMCTSSims simulations as one captured HIP graph
    (after one eager call): same root counts and the same numpy RNG stream as the eager
    search, move for move, with the real network; prints the per-call times."""
    import time

    import azg_amd  # noqa: F401
    from azg_amd.inflexion import InflexionGame
    from azg_amd.mcts import MCTS
    from azg_amd.nnet import NNetWrapper
    from azg_amd.othello import OthelloGame

    args = Args(numMCTSSims=25, cpuct=1, tempThreshold=15)
    game = InflexionGame(7, max_turns=343, max_power=6) if game_name == "inflexion" else OthelloGame(6)
    torch.manual_seed(0)
    w = NNetWrapper(game, device="cuda")
    runs = {}
    for graph in (False, True):
        np.random.seed(7)
        mcts = MCTS(w, args, graph=graph)
        g = game.restarted()
        counts, times = [], []
        for m in range(8):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            pi = mcts.getActionProb(g, temp=1)
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
            counts.append(mcts._engine.root_counts(0).copy())
            g = g.to_next_state(int(np.random.choice(len(pi), p=pi)))
        runs[graph] = (counts, times, np.random.randint(0, 2**32, size=2, dtype=np.uint32).tolist())
        assert (mcts._sims_graph is not None) == graph
    for m, (a, b) in enumerate(zip(runs[False][0], runs[True][0])):
        assert np.array_equal(a, b), m
    assert runs[False][2] == runs[True][2]
    eager, graphed = np.median(runs[False][1][2:]), np.median(runs[True][1][2:])
    print(f"\n{game_name}: getActionProb eager {eager * 1e3:.2f} ms, graph {graphed * 1e3:.2f} ms "
          f"({25 / graphed:.0f} sims/s)")


def test_arena_replays_with_f32_form_where_split_overflows():
    """BatchedArena.playGames with a network that trips the split form's
    range flag replays the games with nnet.replay_form -- the same results and moves
    as an arena run on the replay form from the start."""
    import azg_amd  # noqa: F401
    from azg_amd.arena import BatchedArena
    from azg_amd.inflexion import InflexionGame
    from azg_amd.nnet import InferenceNet, NNetWrapper, replay_form

    net = _overflowing_net()
    game = InflexionGame(7, max_turns=12, max_power=6)
    args = Args(numMCTSSims=3, cpuct=1)
    wrapper = NNetWrapper(game)
    wrapper.nnet = net
    arena = BatchedArena(game, wrapper, args, opponent="greedy")
    assert isinstance(arena.evaluator, InferenceNet) and arena.evaluator.gemm != "f32"
    got = arena.playGames(128)  # 128 leaves a forward: the split-fp16 Winograd form
    assert arena.evaluator.gemm == "f32"
    ref_arena = BatchedArena(game, wrapper, args, opponent="greedy", evaluator=replay_form(net))
    assert got == ref_arena.playGames(128)
    assert np.array_equal(arena.last_moves["actions"], ref_arena.last_moves["actions"])
    assert np.array_equal(arena.last_engine_state["boards"], ref_arena.last_engine_state["boards"])


def test_dropin_pools_engines_and_refolds_trained_weights():
    """a new MCTS per episode (Coach.py:110) reuses the engine and captured graph
    of the last one with the same network (reset: an empty tree, as a new MCTS's dicts), with
    results equal to a fresh engine's; after the network's weights change in place (training)
    the drop-in's evaluator is re-folded, so its counts follow the new weights."""
    import azg_amd  # noqa: F401
    from azg_amd.inflexion import InflexionGame
    from azg_amd.mcts import MCTS
    from azg_amd.nnet import InferenceNet, NNetWrapper

    args = Args(numMCTSSims=25, cpuct=1, tempThreshold=30)
    game = InflexionGame(7, max_turns=343, max_power=6)
    torch.manual_seed(0)
    w = NNetWrapper(game, device="cuda")

    def episode(mcts, seed, moves=4):
        np.random.seed(seed)
        g = game.restarted()
        out = []
        for _ in range(moves):
            pi = mcts.getActionProb(g, temp=1)
            out.append(mcts._engine.root_counts(0).copy())
            g = g.to_next_state(int(np.random.choice(len(pi), p=pi)))
        return out

    m1 = MCTS(w, args)
    c1 = episode(m1, 11)
    eng = m1._engine
    assert m1._sims_graph is not None
    del m1
    m2 = MCTS(w, args)
    c2 = episode(m2, 11)
    assert m2._engine is eng and m2._sims_graph is not None  # pooled engine and graph
    assert all(np.array_equal(a, b) for a, b in zip(c1, c2))
    del m2
    with torch.no_grad():  # "training": the weights move in place
        w.nnet.fc3.weight.mul_(3.0)
        w.nnet.conv2.weight.add_(0.01)
    m3 = MCTS(w, args)
    c3 = episode(m3, 11)
    assert m3._engine is eng
    w_ref = NNetWrapper(game, device="cuda")
    w_ref.nnet.load_state_dict(w.nnet.state_dict())
    w_ref.azg_evaluator = InferenceNet(w_ref.nnet.eval(), conv="miopen", gemm="f32")
    c_ref = episode(MCTS(w_ref, args), 11)
    assert all(np.array_equal(a, b) for a, b in zip(c3, c_ref))
    assert not all(np.array_equal(a, b) for a, b in zip(c1, c3))
