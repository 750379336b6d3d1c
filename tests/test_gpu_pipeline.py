"""GPU consumers of the hot path: the training
examples built by azg_examples, the device-resident trainer, the learn loop,
and the batched Arena (MCTSPlayer vs Random/Greedy) against the reference's
own arena games (tests/golden/arena_*.json.gz)."""
import numpy as np
import pytest
import torch

import oracle_lib as ol

pytestmark = pytest.mark.gpu


class Args(dict):
    __getattr__ = dict.__getitem__


def _cpu_examples(game, rec, label_mode):
    from azg_amd.coach import examples_from_record
    ex = []
    for i in range(len(rec["moves"])):
        ex += examples_from_record(game, rec["actions"][i], rec["temps"][i], rec["counts"][i],
                                   int(rec["moves"][i]), label_mode)
    return ex


def _assert_same(gpu, cpu):
    assert len(gpu) == len(cpu)
    b = np.array([e[0] for e in cpu], np.int64)
    p = np.array([e[1] for e in cpu], np.float64).astype(np.float32)
    v = np.array([e[2] for e in cpu], np.float64).astype(np.float32)
    assert np.array_equal(gpu.planes.cpu().numpy().astype(np.int64), b)
    assert np.array_equal(gpu.pis.cpu().numpy(), p)
    assert np.array_equal(gpu.vs.cpu().numpy(), v)


@pytest.mark.parametrize("game_name,n,max_turns,temp_threshold", [("inflexion", 7, 40, 30),
                                                                  ("inflexion", 7, 60, 5),
                                                                  ("othello", 6, 0, 15)])
@pytest.mark.parametrize("label_mode", ["reference", "per_move"])
def test_examples_match_host_pipeline(game_name, n, max_turns, temp_threshold, label_mode):
    """azg_examples (replay + 36/8 symmetry forms + labels on the GPU) equals the
    host restatement of Coach.py:74-90, which tests/test_examples_cpu.py pins to
    the reference's example hashes."""
    import azg_amd  # noqa: F401
    from azg_amd.engine import SelfPlayEngine
    from azg_amd.examples import engine_examples
    from azg_amd.inflexion import InflexionGame
    from azg_amd.othello import OthelloGame
    kw = dict(max_turns=max_turns) if game_name == "inflexion" else {}
    eng = SelfPlayEngine(6, sims=12, temp_threshold=temp_threshold, game=game_name, n=n, seed_base=17, **kw)
    eng.play()
    rec = eng.read_moves()
    game = InflexionGame(7, max_turns=max_turns, max_power=6) if game_name == "inflexion" else OthelloGame(n)
    cpu = _cpu_examples(game, rec, label_mode)
    gpu = engine_examples(eng, temp_threshold, label_mode, maxlen=10**9)
    _assert_same(gpu, cpu)
    # deque(maxlen) window: the last maxlen examples
    k = len(cpu) // 3 + 5
    win = engine_examples(eng, temp_threshold, label_mode, maxlen=k)
    _assert_same(win, cpu[-k:])
    eng.close()


def test_examples_from_gathered_int16_records_and_bad_record():
    import azg_amd  # noqa: F401
    from azg_amd import _lib
    from azg_amd.dist import engine_records
    from azg_amd.engine import SelfPlayEngine
    from azg_amd.examples import engine_examples, examples_from_records
    eng = SelfPlayEngine(4, sims=8, max_turns=30, seed_base=5)
    eng.play()
    ref = engine_examples(eng, 30, maxlen=10**9)
    moves, actions, counts = engine_records(eng)
    m = int(moves.max())
    got = examples_from_records("inflexion", 7, 30, 30, moves.clone(), actions[:, :m].clone(),
                                counts[:, :m].to(torch.int16), maxlen=10**9)
    assert torch.equal(got.planes, ref.planes) and torch.equal(got.pis, ref.pis) and torch.equal(got.vs, ref.vs)
    bad = actions[:, :m].clone()
    bad[1, 3] = bad[1, 2]  # repeating the last move: its spawn cell is taken / spread origin emptied
    with pytest.raises(_lib.AzgError):
        examples_from_records("inflexion", 7, 30, 30, moves.clone(), bad, counts[:, :m].clone(), maxlen=100)
    eng.close()


@pytest.mark.parametrize("name", ["arena_random", "arena_greedy", "arena_mcts"])
def test_batched_arena_matches_reference(name):
    """Every arena game (MCTSPlayer with the stub evaluator vs the reference's
    RandomPlayer / GreedyPlayer / a second MCTSPlayer with its own sims and cpuct,
    reference colour order) move for move."""
    import azg_amd  # noqa: F401
    from azg_amd.arena import BatchedArena
    from azg_amd.inflexion import InflexionGame
    data = ol.load_json(f"{name}.json.gz")
    cfg, games = data["config"], data["games"]
    game = InflexionGame(7, max_turns=cfg["max_turns"], max_power=6)
    args = Args(numMCTSSims=cfg["sims"], cpuct=cfg["cpuct"])
    if cfg["opponent"] == "mcts":
        arena = BatchedArena(game, "stub", args, opponent="stub", seed_base=cfg["seed_base"],
                             opponent_args=Args(numMCTSSims=cfg["opp_sims"], cpuct=cfg["opp_cpuct"]))
    else:
        arena = BatchedArena(game, "stub", args, opponent=cfg["opponent"], seed_base=cfg["seed_base"])
    one, two, draws = arena.playGames(cfg["num"])
    rec = arena.last_moves
    for i, gm in enumerate(games):
        n = int(rec["moves"][i])
        assert rec["actions"][i, :n].tolist() == gm["actions"], i
    assert one == sum(g["red_wins"] for g in games)
    assert two == sum(g["blue_wins"] for g in games)
    assert draws == sum(g["draws"] for g in games)


def test_batched_arena_two_networks():
    """Net against net (two NNetWrappers of different seeds): every game ends, the records of
    the two engines agree, the results add up, and swapping the networks' colours swaps
    which side searches with which network (the totals stay a partition of the games)."""
    import azg_amd  # noqa: F401
    from azg_amd.arena import BatchedArena
    from azg_amd.inflexion import InflexionGame
    from azg_amd.nnet import NNetWrapper
    game = InflexionGame(7, max_turns=40, max_power=6)
    torch.manual_seed(1)
    w1 = NNetWrapper(game, dict(num_channels=32), device="cuda")
    torch.manual_seed(2)
    w2 = NNetWrapper(game, dict(num_channels=32), device="cuda")
    args = Args(numMCTSSims=8, cpuct=1)
    arena = BatchedArena(game, w1, args, opponent=w2, opponent_args=Args(numMCTSSims=4, cpuct=1.0))
    one, two, draws = arena.playGames(6)
    assert one + two + draws == 6
    st = arena.last_engine_state
    assert int(st["active"].sum()) == 0
    rec = arena.last_moves
    assert (rec["moves"] > 0).all() and (rec["moves"] <= 41).all()
    rb = arena.last_opponent_moves
    assert np.array_equal(rec["moves"], rb["moves"]) and np.array_equal(rec["actions"], rb["actions"])
    with pytest.raises(ValueError):
        BatchedArena(game, w1, args, opponent="minimax")


def test_train_examples_gpu_matches_list_trainer(monkeypatch):
    """NNetWrapper.train_examples (batch gathered on the device) vs the reference
    trainer's list conversion (NNet.py:52-56), both on the GPU."""
    import azg_amd  # noqa: F401
    from azg_amd.coach import examples_from_record
    from azg_amd.examples import ExampleSet
    from azg_amd.inflexion import InflexionGame
    from azg_amd.nnet import NNetWrapper
    game = InflexionGame(7, max_turns=30, max_power=6)
    o = ol.episode(7, 30, 8, 1.0, 10, 3)
    ex = examples_from_record(game, o["actions"], o["temps"], o["counts"], o["moves"])[:300]
    # One SGD step (Adam's g/sqrt(v) turns the GPU backward's summation-order noise
    # on near-zero gradients into full-size steps, and further steps compound it):
    # the comparison is about the sampled batch and the loss, which are identical
    # bit for bit on the CPU (test_pipeline_cpu.py)
    monkeypatch.setattr(NNetWrapper, "_adam", lambda self: torch.optim.SGD(self.nnet.parameters(), lr=1e-3))
    args = dict(epochs=1, batch_size=256, num_channels=16, dropout=0.0)
    nets = []
    for path in ("list", "tensor"):
        torch.manual_seed(0)
        w = NNetWrapper(game, args, device="cuda")
        np.random.seed(11)
        if path == "list":
            w.train(ex)
        else:
            w.train_examples(ExampleSet.from_list(ex, "cuda"))
        nets.append(w.nnet.state_dict())
    for k in nets[0]:
        torch.testing.assert_close(nets[0][k], nets[1][k], rtol=1e-4, atol=1e-5)


def test_fused_adam_matches_foreach_adam():
    """fused_adam=True (opt-in, one kernel per step) applies the update of the
    reference's torch.optim.Adam() (NNet.py:39): one step on the same batch.  Adam's
    first step is lr * g / (|g| + eps); where |g| is near eps the two forms round
    differently (as the GPU backward's summation order already does), so the match is
    checked where the gradient dominates eps (|step| > 0.9 lr), and the bound |step| <= lr
    everywhere."""
    import azg_amd  # noqa: F401
    from azg_amd.coach import examples_from_record
    from azg_amd.examples import ExampleSet
    from azg_amd.inflexion import InflexionGame
    from azg_amd.nnet import NNetWrapper
    game = InflexionGame(7, max_turns=30, max_power=6)
    o = ol.episode(7, 30, 8, 1.0, 10, 3)
    ex = ExampleSet.from_list(examples_from_record(game, o["actions"], o["temps"], o["counts"], o["moves"]), "cuda")
    lr = 1e-3  # torch.optim.Adam's default, as in the reference
    nets = []
    for fused in (False, True):
        torch.manual_seed(0)
        w = NNetWrapper(game, dict(epochs=1, batch_size=len(ex), num_channels=16, dropout=0.0,
                                   fused_adam=fused), device="cuda")
        w0 = {k: v.clone() for k, v in w.nnet.state_dict().items()}
        np.random.seed(11)
        w.train_examples(ex)
        nets.append({k: v - w0[k] for k, v in w.nnet.state_dict().items() if v.is_floating_point()})
    checked = 0
    for k in nets[0]:
        d0, d1 = nets[0][k], nets[1][k]
        if "running" in k:
            torch.testing.assert_close(d0, d1, rtol=1e-5, atol=1e-6)
            continue
        assert d0.abs().max() <= lr * 1.01 and d1.abs().max() <= lr * 1.01, k
        m = d0.abs() > 0.9 * lr
        torch.testing.assert_close(d0[m], d1[m], rtol=1e-3, atol=1e-7)
        checked += int(m.sum())
    assert checked > 1000


def test_bf16_trainer_option_learns():
    """train_dtype="bf16" (opt-in autocast): weights stay f32 and the loss on a fixed
    example set falls over epochs like the f32 trainer's."""
    import azg_amd  # noqa: F401
    from azg_amd.coach import examples_from_record
    from azg_amd.examples import ExampleSet
    from azg_amd.inflexion import InflexionGame
    from azg_amd.nnet import NNetWrapper
    game = InflexionGame(7, max_turns=30, max_power=6)
    o = ol.episode(7, 30, 8, 1.0, 10, 3)
    ex = ExampleSet.from_list(examples_from_record(game, o["actions"], o["temps"], o["counts"], o["moves"]), "cuda")
    for dt in ("f32", "bf16"):
        torch.manual_seed(0)
        w = NNetWrapper(game, dict(epochs=8, batch_size=64, num_channels=32, train_dtype=dt), device="cuda")
        np.random.seed(11)
        losses = w.train_examples(ex).cpu()
        assert torch.isfinite(losses).all()
        assert all(p.dtype == torch.float32 for p in w.nnet.parameters())
        first, last = losses[:4].sum(1).mean(), losses[-4:].sum(1).mean()
        assert last < 0.8 * first, (dt, float(first), float(last))
    with pytest.raises(ValueError):
        NNetWrapper(game, dict(train_dtype="fp8"), device="cuda")._autocast()


def test_learn_loop_small(tmp_path):
    """Coach.learn end to end on the GPU: self-play -> device examples -> train ->
    temp.pth.tar -> arena at iteration 5, with a small net and short games."""
    import os
    import azg_amd  # noqa: F401
    from azg_amd.coach import Coach
    from azg_amd.inflexion import InflexionGame
    from azg_amd.nnet import NNetWrapper
    game = InflexionGame(7, max_turns=12, max_power=6)
    torch.manual_seed(0)
    nnet = NNetWrapper(game, dict(epochs=1, batch_size=64, num_channels=16), device="cuda")
    args = Args(numIters=5, numEps=8, tempThreshold=6, maxlenOfQueue=2000, numMCTSSims=4, cpuct=1,
                arenaCompare=4, checkpoint=str(tmp_path), numItersForTrainExamplesHistory=3,
                saveExamples=True)
    c = Coach(game, nnet, args)
    w0 = {k: v.clone() for k, v in nnet.nnet.state_dict().items()}
    c.learn()
    assert len(c.trainExamplesHistory) == 3
    assert all(len(h) == 2000 for h in c.trainExamplesHistory)
    assert os.path.exists(os.path.join(str(tmp_path), "temp.pth.tar"))
    assert os.path.exists(os.path.join(str(tmp_path), "checkpoint_4.pth.tar.examples"))
    assert any(not torch.equal(w0[k], v) for k, v in nnet.nnet.state_dict().items())
    assert set(c.last_pit) == {"random", "greedy"} and all(sum(r) == 4 for r in c.last_pit.values())
    assert torch.isfinite(c.last_losses).all()


@pytest.mark.parametrize("game_name,n", [("inflexion", 7), ("othello", 6)])
def test_selfplay_slots_refill_same_examples(game_name, n):
    """Coach.selfplay_examples with args.selfplaySlots = 5 < numEps (continuous
    batching through azg_refill) gives exactly the examples of one slot per game."""
    import azg_amd  # noqa: F401
    from azg_amd.coach import Coach
    from azg_amd.inflexion import InflexionGame
    from azg_amd.othello import OthelloGame
    game = InflexionGame(7, max_turns=30, max_power=6) if game_name == "inflexion" else OthelloGame(n)
    base = dict(numEps=13, tempThreshold=10, maxlenOfQueue=10**9, numMCTSSims=8, cpuct=1)
    full = Coach(game, "stub", Args(base)).selfplay_examples(13, first_game=40)
    slim = Coach(game, "stub", Args(base, selfplaySlots=5)).selfplay_examples(13, first_game=40)
    assert len(full) == len(slim) > 0
    assert torch.equal(full.planes, slim.planes)
    assert torch.equal(full.pis, slim.pis)
    assert torch.equal(full.vs, slim.vs)
