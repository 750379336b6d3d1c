"""Data-parallel trainer (ddp.train_examples_dp) at world size 2, gloo, CPU.

The reference trains on one device (inflexion/pytorch/NNet.py:36-76).  Split over two
ranks -- each batch's halves, whole-batch BatchNorm statistics through a differentiable
all-reduce, one gradient all-reduce per step -- the trainer must give the reference
trainer's run (tests/golden/train_golden.json.gz, the dropout-0 run) within the tolerance
of the single-device GPU trainer (tests/test_gpu_train.py: the sums run in another order),
leave numpy's stream where the reference leaves it, and keep the two ranks' weights
bitwise equal (both take the same Adam step on the same all-reduced gradient).  At world
size 1 train_examples is the single-process trainer (tests/test_train_golden.py: bit-equal).
"""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _proj(sd, proj_seed):
    rs = np.random.RandomState(proj_seed)
    out = {}
    for k, v in sd.items():
        f = v.detach().cpu().double().numpy().ravel()
        out[k] = rs.standard_normal((4, f.size)) @ f if f.size else np.zeros(4)
    return out


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        import azg_amd  # noqa: F401
        from azg_amd.examples import ExampleSet
        from azg_amd.nnet import NNetWrapper
        from test_train_golden import golden, reference_examples
        g = golden()
        c = g["config"]
        game, ex = reference_examples(c)
        torch.manual_seed(c["init_seed"])
        w = NNetWrapper(game, dict(num_channels=c["num_channels"], epochs=c["epochs"], dropout=0.0), device="cpu")
        # only rank 0's stream is the reference's: the trainer must draw every batch from it
        np.random.seed(c["batch_seed"] if rank == 0 else 12345)
        losses = w.train_examples(ExampleSet.from_list(ex, "cpu"), group=dist.group.WORLD).numpy()
        sd = {k: v.detach().cpu().numpy().copy() for k, v in w.nnet.state_dict().items()}
        q.put((rank, {"losses": losses, "sd": sd, "rng_pos": int(np.random.get_state()[2]),
                      "rng_next": np.random.randint(0, 2**31, size=4).tolist()}))
    finally:
        dist.destroy_process_group()


def test_data_parallel_trainer_world2():
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_train_golden import golden
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    g = golden()
    c, r = g["config"], g["runs"]["nodropout"]
    # the ranks hold bitwise equal weights and the same numpy stream (rank 0's)
    for k in res[0]["sd"]:
        assert np.array_equal(res[0]["sd"][k], res[1]["sd"][k]), k
    assert res[0]["rng_pos"] == res[1]["rng_pos"] == r["rng_pos"]
    assert res[0]["rng_next"] == res[1]["rng_next"]
    assert np.array_equal(res[0]["losses"], res[1]["losses"])
    # the reference trainer's run, within the single-device GPU trainer's tolerance
    losses = res[0]["losses"].astype(np.float64)
    np.testing.assert_allclose(losses[:2], np.array(r["losses"][:2]), rtol=2e-5)
    np.testing.assert_allclose(losses, np.array(r["losses"]), rtol=2e-3)
    final = _proj({k: torch.from_numpy(v) for k, v in res[0]["sd"].items()}, c["proj_seed"])
    for k in ("conv2.weight", "conv3.weight", "conv4.weight", "fc1.weight", "fc2.weight", "fc3.weight"):
        d_ref = np.array(r["final"][k]["proj"]) - np.array(r["init"][k]["proj"])
        d_dp = final[k] - np.array(r["init"][k]["proj"])
        np.testing.assert_allclose(d_dp, d_ref, rtol=5e-2, atol=5e-2 * float(np.abs(d_ref).max()), err_msg=k)
    # BatchNorm running variances are the whole batch's (not a half's).  (The running means
    # follow the conv / fc biases before them, whose gradient the BatchNorm cancels, so Adam
    # moves them by rounding-noise-driven +-lr steps -- tests/test_gpu_train.py.)
    for k in final:
        if "running_var" in k:
            np.testing.assert_allclose(final[k], np.array(r["final"][k]["proj"]), rtol=1e-3,
                                       atol=1e-3 * float(np.abs(r["final"][k]["proj"]).max()), err_msg=k)
        if k.endswith("num_batches_tracked"):
            assert int(res[0]["sd"][k]) == int(r["final"][k]["sum"]), k


def _dropout_worker(rank, world, port, q):
    """Train with the reference's dropout 0.3 and record every dropout mask this rank draws."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        import torch.nn.functional as F
        import azg_amd  # noqa: F401
        import azg_amd.nnet as nnet_mod
        from azg_amd.examples import ExampleSet
        from azg_amd.nnet import NNetWrapper
        from test_train_golden import golden, reference_examples
        c = golden()["config"]
        game, ex = reference_examples(c)
        torch.manual_seed(c["init_seed"])  # every rank: the same torch generators, as under torchrun
        w = NNetWrapper(game, dict(num_channels=c["num_channels"], epochs=1, dropout=0.3), device="cpu")
        masks = []
        orig = F.dropout

        def recording_dropout(x, p=0.5, training=True, inplace=False):
            m = orig(torch.ones_like(x), p, training)
            masks.append((m != 0).numpy().copy())
            return x * m
        nnet_mod.F.dropout = recording_dropout
        try:
            np.random.seed(c["batch_seed"])
            before = torch.get_rng_state()
            w.train_examples(ExampleSet.from_list(ex, "cpu"), group=dist.group.WORLD)
        finally:
            nnet_mod.F.dropout = orig
        sd = {k: v.detach().cpu().numpy().copy() for k, v in w.nnet.state_dict().items()}
        q.put((rank, {"masks": masks, "sd": sd,
                      "rng_restored": rank != 0 and torch.equal(torch.get_rng_state(), before)}))
    finally:
        dist.destroy_process_group()


def test_data_parallel_dropout_masks_differ_across_ranks():
    """with dropout > 0 each rank's slice gets its own masks (the reference draws an
    independent mask per sample of the whole batch), while the weights stay bitwise equal."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dropout_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    m0, m1 = res[0]["masks"], res[1]["masks"]
    assert len(m0) == len(m1) > 0
    for a, b in zip(m0, m1):
        assert a.shape == b.shape
        assert not np.array_equal(a, b)
        assert 0.6 < a.mean() < 0.8 and 0.6 < b.mean() < 0.8  # keep probability 0.7
    for k in res[0]["sd"]:
        assert np.array_equal(res[0]["sd"][k], res[1]["sd"][k]), k
    assert res[1]["rng_restored"]  # the caller's generator state is restored after training
