"""The drop-in MCTS's idle-engine pool: bounded per key and in all (LRU), and an
evaluator's entries dropped when its module is garbage-collected.  Fake engines, no GPU."""
import gc

import torch

import azg_amd  # noqa: F401
import azg_amd.mcts as m


class FakeEngine:
    closed = []

    def __init__(self, name):
        self.name = name

    def close(self):
        FakeEngine.closed.append(self.name)


def _reset():
    m._POOL.clear()
    m._POOL_ORDER.clear()
    FakeEngine.closed = []


def test_pool_bounds_and_lru():
    _reset()
    for i in range(3):  # per key at most _POOL_MAX
        m._pool_put((1, "a"), (FakeEngine(f"a{i}"), None, 0, False))
    assert len(m._POOL[(1, "a")]) == m._POOL_MAX and FakeEngine.closed == ["a2"]
    for i in range(4):  # in all at most _POOL_TOTAL_MAX: the least recently released go first
        m._pool_put((2, f"k{i}"), (FakeEngine(f"k{i}"), None, 0, False))
    assert len(m._POOL_ORDER) == m._POOL_TOTAL_MAX
    assert FakeEngine.closed == ["a2", "a0", "a1"] and (1, "a") not in m._POOL
    got = m._pool_get((2, "k0"))
    assert got[0].name == "k0" and (2, "k0") not in m._POOL and len(m._POOL_ORDER) == 3
    assert m._pool_get((9, "none")) is None
    m.clear_pool()
    assert not m._POOL and not m._POOL_ORDER
    _reset()


def test_pool_entries_dropped_with_the_module():
    _reset()
    mod = torch.nn.Linear(2, 2)
    ev_id = 12345
    import weakref
    weakref.finalize(mod, m._drop_pooled, ev_id)
    m._pool_put((ev_id, "x"), (FakeEngine("x"), None, 0, False))
    m._pool_put((7, "y"), (FakeEngine("y"), None, 0, False))
    del mod
    gc.collect()
    assert FakeEngine.closed == ["x"] and (ev_id, "x") not in m._POOL and (7, "y") in m._POOL
    assert all(k[0] != ev_id for k in m._POOL_ORDER)
    _reset()
