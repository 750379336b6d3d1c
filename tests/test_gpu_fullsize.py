"""The engine against the oracle at the benchmarked sizes (4096 games per GPU).

Every other parity test runs <= 96 slots; these run BASELINE.json's configs at
full size with the hash evaluator (bit-exact) and compare 32 slots spread over
[0, 4096) -- slot 4095 included -- with the oracle's episode of the same game
index (oracle/oracle.c, pinned to the reference's MCTS.py:62-145 semantics by
tests/test_oracle_golden.py): visit counts and actions of every move played,
and each slot's numpy RNG position after them.

At C3 (100 sims) the node pool is 16 * 100 + 128 = 1728 nodes per game, so the
node_P / node_N / node_Q arrays hold 4096 * 1728 * 384 = 2.72e9 elements: past
2^31, every 64-bit index path of the kernels is exercised.
"""
import numpy as np
import pytest

import oracle_lib as ol

pytestmark = pytest.mark.gpu

G = 4096
SLOTS = sorted(set(np.linspace(0, G - 1, 32).astype(int).tolist()) | {1, G - 2})


@pytest.mark.parametrize("name,game,n,sims,moves,max_turns", [
    ("C4", "inflexion", 7, 25, 5, 343),
    ("C3", "inflexion", 7, 100, 3, 343),
    ("C5", "othello", 8, 200, 2, 0),
])
def test_full_size_vs_oracle(name, game, n, sims, moves, max_turns):
    import azg_amd  # noqa: F401
    from azg_amd.engine import SelfPlayEngine

    e = SelfPlayEngine(G, sims=sims, cpuct=1, temp_threshold=30, max_turns=max_turns or 343, seed_base=0,
                       first_game=0, evaluator="stub", game=game, n=n, max_moves=moves)
    if name == "C3":  # the default pool (azg_capi.cpp: 16 sims + 128 nodes) crosses 2^31 elements
        assert e.cfg.node_capacity == 0 and G * (16 * sims + 128) * 384 > 2**31
    for _ in range(moves):
        e.move()
    st = e.stats()
    assert st["error"] == 0
    rec = e.read_moves()
    kind = ol.OTHELLO if game == "othello" else ol.INFLEXION
    for s in SLOTS:
        o = ol.episode(n, max_turns, sims, 1, 30, s, max_moves=moves, kind=kind)
        m = min(o["moves"], moves)
        assert rec["moves"][s] == m, (name, s)
        assert np.array_equal(rec["actions"][s, :m], o["actions"][:m]), (name, s)
        assert np.array_equal(rec["counts"][s, :m], o["counts"][:m]), (name, s)
        assert e.get_rng(s)[1] == o["rng_pos"], (name, s)
    e.close()
