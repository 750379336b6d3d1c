"""Builder-authored Othello plugin (no reference implementation exists).

Rules pinned by the standard 8x8 Othello perft counts (passes count as moves)
and by agreement with the independent C restatement in oracle/oracle.c."""
import numpy as np

import azg_amd  # noqa: F401
from azg_amd.flags import GameOutcome, PlayerColour
from azg_amd.othello import OthelloGame

PERFT8 = [1, 4, 12, 56, 244, 1396, 8200]


def perft(g, d):
    if d == 0 or g.outcome != GameOutcome.ONGOING:
        return 1
    return sum(perft(g.to_next_state(a), d - 1) for a in np.nonzero(g.valid_actions_mask())[0])


def test_perft_8x8():
    g = OthelloGame(8)
    for d in range(5):
        assert perft(g, d) == PERFT8[d]


def test_api_shapes_and_symmetries():
    g = OthelloGame(6)
    assert g.max_actions == 37 and g.policy_shape == (1, 1, 37)
    p = g.to_planes()
    assert p.shape == (2, 6, 6) and p.sum() == 4
    syms = g.symmetries(p)
    assert len(syms) == 8 and all(s.sum() == 4 for s in syms)
    pi = np.arange(37).reshape(g.policy_shape)
    ps = g.symmetries(pi)
    assert all(s.reshape(-1)[36] == 36 for s in ps)
    assert sorted(ps[3].reshape(-1)[:36].tolist()) == list(range(36))


def test_pass_and_end():
    b = np.zeros((4, 4), dtype=int)
    b[0, 0], b[0, 1] = 1, -1           # RED can capture by playing (0,2)
    g = OthelloGame(4, board=b.copy())
    v = g.valid_actions_mask()
    assert v[2] == 1 and v[16] == 0
    g2 = g.to_next_state(2)
    assert g2.outcome == GameOutcome.LOST and g2.player == PlayerColour.BLUE  # BLUE to move, no pieces


def _perft_c(g, d):
    import ctypes
    import oracle_lib as ol
    if d == 0 or g.outcome != 0:
        return 1
    L = ol.lib()
    valid = np.zeros(65, np.uint8)
    L.orc_valid_mask(ctypes.byref(g), ol.ptr(valid, ctypes.c_uint8))
    tot = 0
    for a in np.nonzero(valid[:g.n * g.n + 1])[0]:
        h = ol.OrcGame()
        ctypes.memmove(ctypes.byref(h), ctypes.byref(g), ctypes.sizeof(g))
        assert L.orc_apply(ctypes.byref(h), int(a)) == 0
        tot += _perft_c(h, d - 1)
    return tot


def test_oracle_othello_perft_and_plugin_agree():
    import ctypes
    import oracle_lib as ol
    g = ol.OrcGame()
    ol.lib().orc_othello_init(ctypes.byref(g), 8)
    assert [_perft_c(g, d) for d in range(6)] == PERFT8[:6]
    # random playouts: C oracle and Python plugin step identically
    rs = np.random.RandomState(9)
    for n in (6, 8):
        for _ in range(20):
            py = OthelloGame(n)
            c = ol.OrcGame()
            ol.lib().orc_othello_init(ctypes.byref(c), n)
            while py.outcome == GameOutcome.ONGOING:
                v = py.valid_actions_mask()
                vc = np.zeros(65, np.uint8)
                ol.lib().orc_valid_mask(ctypes.byref(c), ol.ptr(vc, ctypes.c_uint8))
                assert np.array_equal(v, vc[:n * n + 1])
                a = int(rs.choice(np.nonzero(v)[0]))
                py = py.to_next_state(a)
                ol.lib().orc_apply(ctypes.byref(c), a)
                assert list(c.board)[:n * n] == py._board.ravel().tolist()
                assert ol.OUTCOME_VALUE[c.outcome] == py.outcome.value


def test_oracle_dihedral_matches_plugin():
    import oracle_lib as ol
    from azg_amd.othello import dihedral_source
    for n in (6, 8):
        for k in range(8):
            src = np.zeros(n * n, np.int32)
            import ctypes
            ol.lib().orc_dihedral_gather(n, k, ol.ptr(src, ctypes.c_int))
            rr, qq = dihedral_source(n, k)
            assert src.tolist() == (rr * n + qq).ravel().tolist()


import pytest  # noqa: E402


@pytest.mark.parametrize("name", ["othello6", "othello8", "othello8_s200"])
def test_oracle_othello_episodes_match_reference_search(name):
    """The reference MCTS/Coach driven with this Othello plugin (golden traces)
    vs the C oracle: bit-exact visit counts, actions, expansions, RNG."""
    import oracle_lib as ol
    data = ol.load_json(f"mcts_{name}.json.gz")
    cfg = data["config"]
    for ep in data["episodes"]:
        n = cfg["n"]
        got = ol.episode(n, 0, cfg["sims"], cfg["cpuct"], cfg["temp_threshold"], ep["seed"], kind=ol.OTHELLO)
        assert got["moves"] == ep["n_moves"]
        for m, mv in enumerate(ep["moves"]):
            assert np.array_equal(got["counts"][m], ol.golden_counts(mv, n * n + 1)), (ep["seed"], m)
            assert got["actions"][m] == mv["action"]
        assert got["expansions"] == ep["expansions"] and got["nodes"] == ep["nodes"]
        assert got["rng_pos"] == ep["rng_pos"] and got["rng_next"] == ep["rng_next"]
        assert ol.OUTCOME_VALUE[got["final_outcome"]] == ep["final_outcome"]


def test_othello_examples_from_records_match_reference():
    import hashlib
    import oracle_lib as ol
    from azg_amd.coach import examples_from_record
    data = ol.load_json("mcts_othello6.json.gz")
    cfg = data["config"]
    for ep in data["episodes"][:6]:
        o = ol.episode(cfg["n"], 0, cfg["sims"], cfg["cpuct"], cfg["temp_threshold"], ep["seed"], kind=ol.OTHELLO)
        ex = examples_from_record(OthelloGame(cfg["n"]), o["actions"], o["temps"], o["counts"], o["moves"])
        assert len(ex) == ep["n_examples"]
        assert hashlib.sha256(np.array([e[1] for e in ex], np.float64).tobytes()).hexdigest() == ep["policy_sha256"]
        assert hashlib.sha256(np.array([e[0] for e in ex], np.int64).tobytes()).hexdigest() == ep["board_sha256"]
