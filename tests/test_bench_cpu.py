"""bench.py's algorithmic byte and FLOP models (no GPU): the per-leaf figures DESIGN.md
quotes and the roofline fields are priced with."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402


def test_direct_net_flops_match_survey():
    total, conv234 = bench.net_flops(7, 4, 343)
    assert round(total / 1e6, 1) == 404.3 and round(conv234 / 1e6, 1) == 391.6


def test_winograd_gemm_flops():
    # (11^2 + 7^2 + 5^2) transformed points x 2 x 512^2 per leaf
    assert bench.winograd_flops(7) == (121 + 49 + 25) * 2 * 512 * 512


def test_transform_bytes():
    tb = bench.transform_bytes(7, 4)
    assert tb["first"] == 4 * 49 * 4 + 121 * 512 * 4
    assert tb["mid"] == (121 + 49) * 512 * 4 + (49 + 25) * 512 * 4
    assert tb["out"] == 25 * 512 * 4 + 9 * 512 * 6
    assert tb["total"] == tb["first"] + tb["mid"] + tb["out"] == 827152


def test_tree_bytes_per_expansion():
    # ~4.8 KB per expansion at d = 1.33, A = 87
    b = bench.tree_bytes_per_exp(343, 4 * 49 * 4)
    assert 4700 < b < 4800


def test_presets_are_the_baseline_configs():
    assert bench.PRESETS["C4"] == dict(game="inflexion", n=7, games=4096, sims=25)
    assert bench.PRESETS["C2"]["games"] == 256 and bench.PRESETS["C3"]["sims"] == 100
    assert bench.PRESETS["C5"] == dict(game="othello", n=8, games=4096, sims=200)
