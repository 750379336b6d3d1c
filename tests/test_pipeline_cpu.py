"""Learn-loop pieces that run on the CPU: the device-resident trainer
(NNetWrapper.train_examples) against the reference-format trainer on the same
examples and RNG draws, and the examples file (Coach.py:170-193) round trip."""
import numpy as np
import torch

import azg_amd  # noqa: F401
import oracle_lib as ol
from azg_amd.coach import Coach, examples_from_record
from azg_amd.examples import ExampleSet
from azg_amd.inflexion import InflexionGame
from azg_amd.nnet import NNetWrapper


class Args(dict):
    __getattr__ = dict.__getitem__


def _examples(seed=3, max_turns=30):
    game = InflexionGame(7, max_turns=max_turns, max_power=6)
    o = ol.episode(7, max_turns, 8, 1.0, 10, seed)
    return game, examples_from_record(game, o["actions"], o["temps"], o["counts"], o["moves"])


def test_train_examples_matches_list_trainer():
    """Same Adam steps as NNet.py:36-76 on the same sampled batches: the device
    gather path and the list-conversion path give identical weights."""
    game, ex = _examples()
    args = dict(epochs=2, batch_size=64, num_channels=8)
    nets = []
    for path in ("list", "tensor"):
        torch.manual_seed(0)
        w = NNetWrapper(game, args, device="cpu")
        np.random.seed(11)
        torch.manual_seed(5)  # dropout masks
        if path == "list":
            w.train(ex)
        else:
            losses = w.train_examples(ExampleSet.from_list(ex, "cpu"))
            assert losses.shape == (2 * (len(ex) // 64), 2) and torch.isfinite(losses).all()
        nets.append(w.nnet.state_dict())
    for k in nets[0]:
        assert torch.equal(nets[0][k], nets[1][k]), k


def test_example_set_list_roundtrip():
    game, ex = _examples(seed=4)
    s = ExampleSet.from_list(ex, "cpu")
    assert len(s) == len(ex) and s.planes.shape == (len(ex), 4, 7, 7) and s.pis.shape == (len(ex), 343)
    back = s.to_list()
    for (b0, p0, z0), (b1, p1, z1) in zip(ex, back):
        assert np.array_equal(np.asarray(b0), b1)
        assert np.array_equal(np.asarray(p0, np.float32), np.asarray(p1, np.float32))
        assert float(z0) == z1


def test_examples_file_roundtrip(tmp_path):
    game, ex = _examples(seed=5)
    args = Args(checkpoint=str(tmp_path), maxlenOfQueue=200000,
                load_folder_file=(str(tmp_path), "checkpoint_0.pth.tar"))
    c = Coach(game, "stub", args)
    h = [ExampleSet.from_list(ex[:500], "cpu"), ExampleSet.from_list(ex[500:], "cpu")]
    c.trainExamplesHistory = h
    c.saveTrainExamples(0)
    c2 = Coach(game, "stub", args)
    c2.loadTrainExamples(device="cpu")
    assert c2.skipFirstSelfPlay and len(c2.trainExamplesHistory) == 2
    for a, b in zip(h, c2.trainExamplesHistory):
        assert torch.equal(a.planes, b.planes) and torch.equal(a.pis, b.pis) and torch.equal(a.vs, b.vs)
