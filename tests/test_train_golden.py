"""The trainer against the REFERENCE trainer.

tests/golden/train_golden.json.gz holds the reference NNetWrapper.train
(inflexion/pytorch/NNet.py:36-76: Adam, epochs x len//batch_size batches drawn
with np.random.randint, the two losses of :96-100) run on the examples of one
reference Coach.executeEpisode, with NNet.args shrunk to 32 channels x 2 epochs:
every batch's (l_pi, l_v) and the weights after training (per-tensor sha256,
sums, projections), with the reference's dropout 0.3 and with dropout 0.

On the CPU (one torch thread, as the fixture was made) NNetWrapper.train and
NNetWrapper.train_examples must reproduce the reference bit for bit: same initial
weights, same losses, same final weights (every tensor's sha256, BatchNorm
running statistics included).
"""
import hashlib

import numpy as np
import pytest
import torch

import azg_amd  # noqa: F401
import oracle_lib as ol
from azg_amd.coach import examples_from_record
from azg_amd.examples import ExampleSet
from azg_amd.inflexion import InflexionGame
from azg_amd.nnet import NNetWrapper


def _sha(t):
    return hashlib.sha256(t.detach().cpu().contiguous().numpy().tobytes()).hexdigest()


def golden():
    return ol.load_json("train_golden.json.gz")


def reference_examples(c):
    """The fixture's examples, rebuilt from the oracle's episode (its visit counts and
    actions are the reference's) and checked against the fixture's hashes."""
    game = InflexionGame(7, max_turns=c["max_turns"], max_power=6)
    o = ol.episode(7, c["max_turns"], c["sims"], c["cpuct"], c["temp_threshold"], c["seed"])
    ex = examples_from_record(game, o["actions"], o["temps"], o["counts"], o["moves"])
    return game, ex


@pytest.fixture(scope="module")
def one_thread():
    n = torch.get_num_threads()
    torch.set_num_threads(1)
    yield
    torch.set_num_threads(n)


def test_examples_are_the_fixtures():
    g = golden()
    _, ex = reference_examples(g["config"])
    assert len(ex) == g["n_examples"]
    assert hashlib.sha256(np.array([e[1] for e in ex], np.float64).tobytes()).hexdigest() == \
        g["examples_policy_sha256"]
    assert hashlib.sha256(np.array([e[0] for e in ex], np.int64).tobytes()).hexdigest() == g["examples_board_sha256"]
    assert hashlib.sha256(np.array([e[2] for e in ex], np.float64).tobytes()).hexdigest() == g["examples_z_sha256"]


@pytest.mark.parametrize("run", ["dropout", "nodropout"])
@pytest.mark.parametrize("path", ["train", "train_examples"])
def test_trainer_bit_equal_to_reference(one_thread, run, path):
    g = golden()
    c, r = g["config"], g["runs"][run]
    game, ex = reference_examples(c)
    torch.manual_seed(c["init_seed"])
    w = NNetWrapper(game, dict(num_channels=c["num_channels"], epochs=c["epochs"], dropout=r["dropout"]),
                    device="cpu")
    sd = w.nnet.state_dict()
    assert list(sd) == list(r["init"]), "parameter names / creation order"
    for k, v in sd.items():
        assert _sha(v) == r["init"][k]["sha256"], f"initial {k}"
    np.random.seed(c["batch_seed"])
    torch.manual_seed(c["torch_seed"])
    if path == "train":
        w.train(ex)
    else:
        losses = w.train_examples(ExampleSet.from_list(ex, "cpu")).numpy()
        assert losses.tolist() == [[np.float32(a), np.float32(b)] for a, b in r["losses"]]
    assert int(np.random.get_state()[2]) == r["rng_pos"]
    for k, v in w.nnet.state_dict().items():
        assert _sha(v) == r["final"][k]["sha256"], f"final {k}"


def test_train_full_sensitivity_fixture():
    """tests/golden/train_full_sensitivity.json.gz (the reference trainer at 512 channels rerun from
    initial weights moved by a few ulps, 3 seeds) against train_full_golden.json.gz: the same
    examples and config, initial projections within 1e-6 of the unperturbed run's, first-batch
    losses within 1e-5 -- and the spread it records: Adam's sign-steps make the reference's own
    two-step conv3 update move by more than 5e-2 of its size for one seed (tests/test_gpu_train.py
    holds the GPU trainer to 1.25x this spread where it exceeds 5e-2)."""
    g = ol.load_json("train_full_golden.json.gz")
    s = ol.load_json("train_full_sensitivity.json.gz")
    assert s["config"] == g["config"] and s["n_examples"] == g["n_examples"] and len(s["runs"]) == 3
    r = g["runs"]["nodropout"]
    spread = {}
    for q in s["runs"].values():
        np.testing.assert_allclose(q["losses"][0], r["losses"][0], rtol=1e-5)
        for k, v in q["init"].items():
            a, b = np.array(v["proj"]), np.array(r["init"][k]["proj"])
            assert np.abs(a - b).max() <= 1e-6 * np.abs(b).max() + 1e-9, k
            d_ref = np.array(r["final"][k]["proj"]) - b
            d = np.array(q["final"][k]["proj"]) - a
            spread[k] = max(spread.get(k, 0.0), float(np.abs(d - d_ref).max() / np.abs(d_ref).max()))
    assert spread["conv3.weight"] > 5e-2 and max(v for k, v in spread.items() if k != "conv3.weight") < 5e-2, spread
