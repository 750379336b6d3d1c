"""Training-example pipeline (Coach.py:74-90) from move records, on CPU.

Move records come from the oracle (same records the engine writes); the
examples must hash-match those the reference Coach returned for the same seed,
including its cumulative player-label quirk (Coach.py:79)."""
import hashlib

import numpy as np
import pytest

import azg_amd  # noqa: F401
import oracle_lib as ol
from azg_amd.coach import _label_players, examples_from_record
from azg_amd.inflexion import InflexionGame


def _rle(zs):
    out = []
    for z in zs:
        if out and out[-1][0] == z:
            out[-1][1] += 1
        else:
            out.append([z, 1])
    return out


@pytest.mark.parametrize("name,limit", [("short", 16), ("main", 3)])
def test_examples_from_records_match_reference(name, limit):
    data = ol.load_json(f"mcts_{name}.json.gz")
    cfg = data["config"]
    game = InflexionGame(7, max_turns=cfg["max_turns"], max_power=6)
    for ep in data["episodes"][:limit]:
        o = ol.episode(7, cfg["max_turns"], cfg["sims"], cfg["cpuct"], cfg["temp_threshold"], ep["seed"])
        ex = examples_from_record(game, o["actions"], o["temps"], o["counts"], o["moves"])
        assert len(ex) == ep["n_examples"]
        assert _rle([float(e[2]) for e in ex]) == ep["z_rle"]
        assert hashlib.sha256(np.array([e[1] for e in ex], np.float64).tobytes()).hexdigest() == ep["policy_sha256"]
        assert hashlib.sha256(np.array([e[0] for e in ex], np.int64).tobytes()).hexdigest() == ep["board_sha256"]


def test_label_modes():
    players = [1, -1, 1]
    ref = _label_players(players, "reference")
    # reference list: 36 x p1, then 72 x p2, ... truncated to 108 examples by zip
    assert (ref[:36] == 1).all() and (ref[36:108] == -1).all()
    fixed = _label_players(players, "per_move")
    assert (fixed[:36] == 1).all() and (fixed[36:72] == -1).all() and (fixed[72:] == 1).all()
