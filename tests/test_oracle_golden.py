"""Pin the CPU oracle against fixtures generated from the reference itself.

CPU-only.  Fixtures: tests/golden/* (tests/golden/make_golden.py).
"""
import ctypes

import numpy as np
import pytest

import oracle_lib as ol
from golden.stubnet import stub_eval as stub_eval_np


def test_rng_raw_and_ops():
    for case in ol.load_json("rng_kat.json.gz"):
        r = ol.Rng(case["seed"])
        assert [r.u32() for _ in range(len(case["raw_u32"]))] == case["raw_u32"]
        r = ol.Rng(case["seed"])
        for t, op in enumerate(case["ops"]):
            kind = op[0]
            if kind == "randint":
                assert r.randint(op[1], op[2]) == op[3]
            elif kind == "choice3":
                assert r.randint(0, 3) == op[1]
            elif kind == "random_sample":
                assert r.random_sample() == op[1]
            elif kind == "choice_n":
                assert r.randint(0, op[1]) == op[2]
            elif kind == "choice_p":
                if t % 2:  # the generator drew the weights from the same stream
                    for _ in range(13):
                        r.random_sample()
                assert r.choice_p(np.array(op[1])) == op[2]
            else:
                p = np.zeros(9)
                p[op[1]] = 1.0
                assert r.choice_p(p) == op[2]


def test_symmetry_tables():
    sym = ol.load_json("symmetry.json.gz")
    n = 7
    for k in range(6):
        assert ol.sym_gather(n, k, 0, 0).tolist() == sym["rotate"][k]
    for ax_i, ax in enumerate("rqs"):
        for j in range(7):
            assert ol.sym_gather(n, 0, j, ax_i).tolist() == sym["translate"][ax][j]
    order = [(0, 0)] + [(k, 0) for k in range(1, 6)] + [(k, j) for k in range(1, 6) for j in range(1, 7)]
    assert len(order) == len(sym["symmetries"]) == 36
    for (k, j), want in zip(order, sym["symmetries"]):
        assert ol.sym_gather(n, k, j, 0).tolist() == want


def test_rules_playouts():
    d = dict(np.load(ol.os.path.join(ol.GOLDEN, "rules_kat.npz")))
    L = ol.lib()
    nply = len(d["action"])
    g = ol.OrcGame()
    valid = np.zeros(343, np.uint8)
    planes = np.zeros(4 * 49, np.int32)
    for i in range(nply):
        L.orc_game_init(ctypes.byref(g), 7, int(d["max_turns"][i]))
        for c in range(49):
            g.board[c] = int(d["board"][i][c])
        g.turn = int(d["turn"][i])
        g.player = int(d["player"][i])
        L.orc_valid_mask(ctypes.byref(g), ol.ptr(valid, ctypes.c_uint8))
        assert np.array_equal(np.packbits(valid), d["valid_bits"][i]), i
        L.orc_planes(ctypes.byref(g), ol.ptr(planes, ctypes.c_int32))
        b = d["board"][i].astype(np.int64) * g.player
        assert np.array_equal(planes[:49], (b > 0).astype(np.int32))
        assert np.array_equal(planes[49:98], (b < 0).astype(np.int32))
        assert L.orc_apply(ctypes.byref(g), int(d["action"][i])) == 0
        assert ol.OUTCOME_VALUE[g.outcome] == d["outcome"][i], i
        if i + 1 < nply and d["game"][i + 1] == d["game"][i]:
            assert list(g.board)[:49] == d["board"][i + 1].tolist(), i
    # terminal kinds are all covered by the fixture
    assert set(np.unique(d["outcome"]).tolist()) >= {0.0, 1e-4, -1.0}


def test_pairwise_sum():
    d = dict(np.load(ol.os.path.join(ol.GOLDEN, "pairwise_kat.npz")))
    L = ol.lib()
    for x, n, s in zip(d["x"], d["n"], d["s"]):
        x = np.ascontiguousarray(x, np.float32)
        got = L.orc_pairwise_sum_f32(ol.ptr(x, ctypes.c_float), int(n))
        assert np.float32(got) == s


def test_stub_eval_matches_numpy_spec():
    rs = np.random.RandomState(3)
    for _ in range(200):
        planes = np.zeros((4, 7, 7), np.int64)
        planes[0] = rs.random_sample((7, 7)) < 0.3
        planes[1] = (rs.random_sample((7, 7)) < 0.3) & (planes[0] == 0)
        planes[2] = rs.randint(0, 344)
        planes[3] = rs.randint(0, 2)
        P1, v1 = stub_eval_np(planes, 343)
        P2, v2 = ol.stub_eval(planes)
        assert np.array_equal(P1.view(np.uint32), P2.view(np.uint32))
        assert v1[0] == v2[0]


def _check_episode(cfg, ep, got):
    assert got["moves"] == ep["n_moves"]
    for m, mv in enumerate(ep["moves"]):
        want = ol.golden_counts(mv)
        assert np.array_equal(got["counts"][m], want), f"seed {ep['seed']} move {m}"
        assert got["actions"][m] == mv["action"], f"seed {ep['seed']} move {m}"
        assert got["temps"][m] == mv["temp"]
    assert got["expansions"] == ep["expansions"]
    assert got["nodes"] == ep["nodes"]
    assert ol.OUTCOME_VALUE[got["final_outcome"]] == ep["final_outcome"]
    assert got["final_player"] == ep["final_player"]
    assert got["rng_pos"] == ep["rng_pos"]
    assert got["rng_next"] == ep["rng_next"]


@pytest.mark.parametrize("name", ["short", "main", "pit", "sims100", "deep"])
def test_mcts_episodes_bit_exact(name):
    data = ol.load_json(f"mcts_{name}.json.gz")
    cfg = data["config"]
    for ep in data["episodes"]:
        got = ol.episode(7, cfg["max_turns"], cfg["sims"], cfg["cpuct"], cfg["temp_threshold"], ep["seed"])
        _check_episode(cfg, ep, got)


def test_realnet_fixtures_consistent():
    """The real-network reference traces (make_golden `realnet`) and the reference's own
    sensitivity runs (`sensitivity`) that tests/test_gpu_realnet.py certifies near-ties with."""
    main = ol.load_json("mcts_realnet_main.json.gz")
    assert [e["seed"] for e in main["episodes"]] == list(range(8))
    for ep in main["episodes"]:
        assert ep["n_moves"] == len(ep["moves"]) == 344
        for m, mv in enumerate(ep["moves"]):
            counts = ol.golden_counts(mv)
            assert counts.sum() >= main["config"]["sims"] and counts[mv["action"]] > 0 or mv["temp"] == 1, m
    sens = ol.load_json("realnet_sensitivity.json.gz")
    runs = {(r["kind"], r["eps"], r["seed"]): r["first_divergent_move"] for r in sens["runs"]}
    assert len(runs) == 32
    # the near-ties the reference's own rounding decides: by 1e-7, seed 0 at move
    # 222 and seed 3 at 197; by 1e-6, seed 3 at 197 and seed 4 at 277; no other game moves
    w7 = {s: runs[("weights", 1e-7, s)] for s in range(8)}
    w6 = {s: runs[("weights", 1e-6, s)] for s in range(8)}
    assert w7 == {0: 222, 1: None, 2: None, 3: 197, 4: None, 5: None, 6: None, 7: None}
    assert w6 == {0: None, 1: None, 2: None, 3: 197, 4: 277, 5: None, 6: None, 7: None}
