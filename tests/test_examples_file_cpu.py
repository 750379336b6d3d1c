"""The examples file and the shuffle of Coach.learn (Coach.py:143-149, 170-193) on the CPU:

* examples.shuffle_perm (libazg azg_py_shuffle, host code) against Python's random.shuffle
  itself -- same permutation, same `random` stream position afterwards;
* the manifest format: every window written once, later saves naming the same files (the
  save costs O(new windows)), exact round trip of planes / pis / vs;
* the reference format: export_reference_examples' streamed pickle unpickles to the list of
  deques Coach.py:176 writes (equal tuples, deque maxlen), and a reference-written pickle
  loads through loadTrainExamples.
"""
import os
import pickle
import random
import time
from collections import deque

import numpy as np
import pytest
import torch

import azg_amd  # noqa: F401
import oracle_lib as ol
from azg_amd.coach import Coach, examples_from_record
from azg_amd.examples import (ExampleSet, export_reference_examples, is_manifest, read_examples_file,
                              shuffle_perm, write_manifest)
from azg_amd.inflexion import InflexionGame


class Args(dict):
    __getattr__ = dict.__getitem__


def _examples(seed, max_turns=30):
    game = InflexionGame(7, max_turns=max_turns, max_power=6)
    o = ol.episode(7, max_turns, 8, 1.0, 10, seed)
    return game, examples_from_record(game, o["actions"], o["temps"], o["counts"], o["moves"])


@pytest.mark.parametrize("n", [0, 1, 2, 3, 17, 1000, 65537, 300001])
def test_shuffle_perm_is_random_shuffle(n):
    random.seed(1234 + n)
    random.random()  # a state in the middle of a 624-word block
    st = random.getstate()
    ref = list(range(n))
    random.shuffle(ref)
    after_ref = random.getstate()
    random.setstate(st)
    perm = shuffle_perm(n)
    assert perm.dtype == np.int64 and perm.tolist() == ref
    assert random.getstate() == after_ref
    assert random.random() == (random.setstate(after_ref) or random.random())


def test_shuffle_perm_speed():
    """The 4M-example steady-state history's shuffle: natively well under the interpreter's ~1.8 s."""
    random.seed(0)
    t = time.perf_counter()
    p = shuffle_perm(4_000_000)
    dt = time.perf_counter() - t
    assert len(p) == 4_000_000 and dt < 0.5, dt


def _coach(tmp_path, fmt, name="checkpoint_0.pth.tar"):
    game = InflexionGame(7, max_turns=30, max_power=6)
    args = Args(checkpoint=str(tmp_path), maxlenOfQueue=200000, examplesFormat=fmt,
                load_folder_file=(str(tmp_path), name))
    return Coach(game, "stub", args)


def _same(a, b):
    return torch.equal(a.planes, b.planes) and torch.equal(a.pis, b.pis) and torch.equal(a.vs, b.vs)


def test_manifest_writes_each_window_once(tmp_path):
    _, ex = _examples(seed=5)
    _, ex2 = _examples(seed=6)
    c = _coach(tmp_path, "azg", "checkpoint_1.pth.tar")
    w0, w1, w2 = (ExampleSet.from_list(e, "cpu") for e in (ex[:500], ex[500:], ex2))
    c.trainExamplesHistory = [w0, w1]
    c.saveTrainExamples(0)
    assert c.last_windows_written == 2
    f0 = (tmp_path / "checkpoint_0.pth.tar.examples")
    assert is_manifest(str(f0)) and f0.stat().st_size < 4096
    # the next iteration: the oldest window dropped, a new one appended -> one file written
    c.trainExamplesHistory = [w1, w2]
    c.saveTrainExamples(1)
    assert c.last_windows_written == 1
    assert len(os.listdir(tmp_path / "examples_windows")) == 3
    c2 = _coach(tmp_path, "azg", "checkpoint_1.pth.tar")
    c2.loadTrainExamples(device="cpu")
    assert c2.skipFirstSelfPlay and len(c2.trainExamplesHistory) == 2
    assert all(_same(a, b) for a, b in zip([w1, w2], c2.trainExamplesHistory))
    # loaded windows remember their files: saving the loaded history writes nothing new
    c2.saveTrainExamples(2)
    assert c2.last_windows_written == 0
    # the iteration-0 file still reads back as it was
    assert all(_same(a, b) for a, b in zip([w0, w1], read_examples_file(str(f0), "cpu")))


def test_manifest_exact_for_any_values(tmp_path):
    """Non-integer planes stay f32, dense arbitrary pis and z values come back bit for bit."""
    g = torch.Generator().manual_seed(3)
    E, A = 257, 343
    planes = torch.randn((E, 4, 7, 7), generator=g)
    pis = torch.rand((E, A), generator=g) * (torch.rand((E, A), generator=g) < 0.5)
    vs = torch.tensor([1.0, -1.0, 1e-4, -1e-4, 0.25] * 51 + [1.0, -1.0])
    h = [ExampleSet(planes, pis, vs), ExampleSet(torch.full((3, 4, 7, 7), 343.0), torch.eye(3, A), vs[:3])]
    f = str(tmp_path / "x.examples")
    write_manifest(h, f)
    back = read_examples_file(f, "cpu")
    assert back[0].planes.dtype == torch.float32
    assert all(_same(a, b) for a, b in zip(h, back))


def test_reference_format_export_and_load(tmp_path):
    _, ex = _examples(seed=7)
    c = _coach(tmp_path, "reference")
    h = [ExampleSet.from_list(ex[:300], "cpu"), ExampleSet.from_list(ex[300:], "cpu")]
    c.trainExamplesHistory = h
    c.saveTrainExamples(0)
    fn = str(tmp_path / "checkpoint_0.pth.tar.examples")
    assert not is_manifest(fn)
    with open(fn, "rb") as f:
        hist = pickle.Unpickler(f).load()  # what the reference's loadTrainExamples does (Coach.py:189)
    assert isinstance(hist, list) and len(hist) == 2
    for d, s in zip(hist, h):
        assert isinstance(d, deque) and d.maxlen == 200000
        want = s.to_list()
        assert len(d) == len(want)
        for (b0, p0, z0), (b1, p1, z1) in zip(d, want):
            assert b0.dtype == np.int64 and np.array_equal(b0, b1)
            assert p0 == p1 and type(z0) is type(z1) and z0 == z1
    c2 = _coach(tmp_path, "azg")
    c2.loadTrainExamples(device="cpu")
    assert all(_same(a, b) for a, b in zip(h, c2.trainExamplesHistory))


def test_reference_written_pickle_loads(tmp_path):
    """A file as the reference writes it (Pickler(f).dump of its deques of executeEpisode tuples)."""
    _, ex = _examples(seed=8)
    hist = [deque(ex[:200], maxlen=200000), deque(ex[200:], maxlen=200000)]
    with open(tmp_path / "checkpoint_0.pth.tar.examples", "wb") as f:
        pickle.Pickler(f).dump(hist)
    c = _coach(tmp_path, "azg")
    c.loadTrainExamples(device="cpu")
    assert [len(h) for h in c.trainExamplesHistory] == [200, len(ex) - 200]
    ref = ExampleSet.from_list(ex, "cpu")
    got = ExampleSet.cat(c.trainExamplesHistory)
    assert _same(ref, got)
    # and re-exported in the reference's format it is the same list of tuples
    out = str(tmp_path / "re.examples")
    export_reference_examples(c.trainExamplesHistory, out, 200000)
    with open(out, "rb") as f:
        back = pickle.load(f)
    assert [len(d) for d in back] == [len(d) for d in hist]
