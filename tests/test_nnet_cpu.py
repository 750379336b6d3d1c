"""The leaf network reproduces the reference InflexionNNet (CPU, f32).

Pinned by tests/golden/nnet_golden.npz, generated from the reference NNetWrapper
under torch.manual_seed(0): per-tensor SHA-256 of the random-init state_dict and
64 batch-1 predictions (planes -> P, v)."""
import hashlib
import os

import numpy as np
import pytest
import torch

import azg_amd  # noqa: F401
from azg_amd.nnet import InflexionNNet, NNetWrapper

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "nnet_golden.npz")


def test_state_dict_matches_reference_init():
    d = dict(np.load(G))
    torch.manual_seed(0)
    net = InflexionNNet()
    sd = net.state_dict()
    assert list(sd.keys()) == d["names"].tolist()
    for k, sha in zip(d["names"], d["sha256"]):
        assert hashlib.sha256(sd[str(k)].contiguous().numpy().tobytes()).hexdigest() == sha, k


def test_predict_matches_reference():
    d = dict(np.load(G))
    torch.manual_seed(0)
    w = NNetWrapper(device="cpu")
    for planes, P, v in zip(d["planes"], d["P"], d["v"]):
        p2, v2 = w.predict(planes.astype(np.int64))
        np.testing.assert_allclose(p2, P, rtol=1e-5, atol=1e-7)
        np.testing.assert_allclose(v2[0], v, rtol=1e-5, atol=1e-6)


def test_batched_matches_batch1():
    d = dict(np.load(G))
    torch.manual_seed(0)
    w = NNetWrapper(device="cpu")
    P, v = w.predict_batch(torch.from_numpy(d["planes"].astype(np.float32)))
    np.testing.assert_allclose(P.numpy(), d["P"], rtol=2e-5, atol=1e-7)
    np.testing.assert_allclose(v.numpy(), d["v"], rtol=2e-5, atol=1e-6)


def test_inference_net_matches_reference_net():
    from azg_amd.nnet import InferenceNet
    d = dict(np.load(G))
    torch.manual_seed(0)
    net = InflexionNNet().eval()
    # non-trivial BatchNorm statistics so the folding is exercised
    g = torch.Generator().manual_seed(1)
    for m in net.modules():
        if isinstance(m, (torch.nn.BatchNorm1d, torch.nn.BatchNorm2d)):
            m.running_mean.normal_(0, 0.1, generator=g)
            m.running_var.uniform_(0.5, 1.5, generator=g)
            m.weight.data.uniform_(0.5, 1.5, generator=g)
            m.bias.data.normal_(0, 0.1, generator=g)
    x = torch.from_numpy(d["planes"].astype(np.float32))
    with torch.no_grad():
        lp, v = net(x)
        p2, v2 = InferenceNet(net)(x)
    np.testing.assert_allclose(p2.numpy(), torch.exp(lp).numpy(), rtol=1e-5, atol=1e-8)
    np.testing.assert_allclose(v2.numpy(), v.numpy(), rtol=1e-5, atol=1e-6)


def test_winograd_layout_matches_libazg():
    """The Python mirror of the mixed-tile layout (GEMM grouping, U order) agrees with
    the kernels' own (azg_winograd_layout), and covers each axis exactly."""
    import ctypes
    from azg_amd import _lib
    from azg_amd.nnet import winograd_groups, winograd_points, winograd_seq, winograd_types
    L = _lib.lib()
    assert winograd_seq(7) == [4, 3] and winograd_seq(5) == [5] and winograd_seq(3) == [3]
    assert winograd_seq(8) == [4, 4] and winograd_seq(6) == [3, 3] and winograd_seq(4) == [4]
    assert winograd_points(7) == 121 and winograd_points(5) == 49 and winograd_points(3) == 25
    for h in range(1, 30):
        seq = (ctypes.c_int32 * 16)()
        groups = (ctypes.c_int32 * 4)()
        p = L.azg_winograd_layout(h, seq, groups)
        assert list(seq[:p]) == winograd_seq(h), h
        assert sum(winograd_seq(h)) == max(h, 2), h  # exact cover (h = 1 pads to one 2-tile)
        assert p == max(1, -(-h // 5)), h  # the fewest tiles of side <= 5
        big, small = winograd_types(h)
        assert set(winograd_seq(h)) <= {big, small} and big == small + 1, h
        want = {(ma, mb): n for ma, mb, _, n in winograd_groups(h)}
        for g, (ma, mb) in enumerate(((big, big), (big, small), (small, big), (small, small))):
            assert groups[g] == want.get((ma, mb), 0), (h, g)


@pytest.mark.parametrize("m", [2, 3, 4, 5])
def test_winograd_tables_are_exact(m):
    """The kernels' B^T, A^T (azg_winograd_tables) with nnet.WINOGRAD_G compute the 3-tap
    correlation: A^T [(G g) * (B^T d)] = sum_k g_k d_{i+k}, in f64, for every basis g, d."""
    import ctypes
    from azg_amd import _lib
    from azg_amd.nnet import WINOGRAD_G
    n = m + 2
    bt = (ctypes.c_float * (n * n))()
    at = (ctypes.c_float * (m * n))()
    assert _lib.lib().azg_winograd_tables(m, bt, at) == 0
    BT = np.array(bt[:], np.float64).reshape(n, n)
    AT = np.array(at[:], np.float64).reshape(m, n)
    G = np.array(WINOGRAD_G[m], np.float64)
    for k in range(3):
        for l in range(n):
            g = np.eye(3)[k]
            d = np.eye(n)[l]
            y = AT @ ((G @ g) * (BT @ d))
            want = np.array([1.0 if l == i + k else 0.0 for i in range(m)])
            np.testing.assert_allclose(y, want, atol=1e-12)


def test_split2_operand_blocks():
    """The split GEMM's operand rows (azg.h AZG_WINO_SPLIT2): 32-channel blocks
    [hi(32) | lo(32)], channel j's hi at 64 (j // 32) + j % 32 and its lo 32 further;
    split2_halves inverts split2_rows, and _split_operands("split") lays U^T out so."""
    import torch
    from azg_amd.nnet import _split_operands, _split_u, split2_halves, split2_rows
    hi = torch.arange(3 * 128, dtype=torch.float32).reshape(3, 128).half()
    lo = -hi
    r = split2_rows(hi, lo)
    assert r.shape == (3, 256)
    for j in (0, 31, 32, 77, 127):
        assert r[1, 64 * (j // 32) + j % 32] == hi[1, j] and r[1, 64 * (j // 32) + 32 + j % 32] == lo[1, j]
    h2, l2 = split2_halves(r)
    assert torch.equal(h2, hi) and torch.equal(l2, lo)
    u = torch.randn(2, 64, 256, dtype=torch.float64)  # [points][C][K]
    b, scale = _split_operands(u, "split")
    uh, ul, s2 = _split_u(u)
    bh, bl = split2_halves(b)
    assert scale == s2 and b.shape == (2, 256, 128)
    assert torch.equal(bh, uh.transpose(1, 2)) and torch.equal(bl, ul.transpose(1, 2))


def _rescaled(net, layer, factor, nxt):
    """net with BatchNorm `layer`'s gamma and beta times `factor` and the next layer's weights
    divided by it: the same function (exactly, for a power of two), small activations between."""
    import copy
    out = copy.deepcopy(net)
    with torch.no_grad():
        bn = getattr(out, layer)
        bn.weight.mul_(factor)
        bn.bias.mul_(factor)
        getattr(out, nxt).weight.div_(factor)
    return out


@pytest.mark.parametrize("layer,nxt", [("bn2", "conv3"), ("bn4", "fc1"), ("fc_bn1", "fc2")])
def test_activation_scales_are_exact(layer, nxt):
    """InferenceNet's power-of-two activation scales (nnet.act_exponent) change no f32 result:
    a network whose BatchNorm shrinks one layer's activations by 2^-10 (the next layer's weights
    grown by 2^10: the same function, exactly) is evaluated with that layer rescaled by 2^11 and
    gives bit-identical P, v to the original network's inference form (f32 arithmetic is
    invariant under exact power-of-two scalings); a random-init network is left unscaled."""
    from azg_amd.nnet import InferenceNet
    torch.manual_seed(0)
    net = InflexionNNet().eval()
    small = _rescaled(net, layer, 2.0 ** -10, nxt).eval()
    a, b = InferenceNet(net), InferenceNet(small)
    assert set(a.act_exp.values()) == {0}
    key = {"bn2": 2, "bn4": 4, "fc_bn1": "fc1"}[layer]
    assert b.act_exp[key] == 11 and all(v == 0 for k, v in b.act_exp.items() if k != key)
    x = (torch.rand(16, 4, 7, 7, generator=torch.Generator().manual_seed(1)) < 0.3).float()
    with torch.no_grad():
        pa, va = a(x)
        pb, vb = b(x)
        lp, vr = small(x)
    assert torch.equal(pa, pb) and torch.equal(va, vb)
    torch.testing.assert_close(pb, torch.exp(lp), rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(vb.reshape(-1), vr.reshape(-1), rtol=1e-5, atol=1e-6)


def test_trained_network_fixture():
    """tests/golden/trained_net.npz (make_golden.py trained_net: the reference NNetWrapper trained
    by its own NNet.train on three of its own self-play episodes) loads into InflexionNNet, whose
    batch-1 predict reproduces the reference's on the fixture's 64 positions; the training took:
    the priors at the initial position are far from the random-init network's near-uniform ones."""
    import oracle_lib as ol
    d = np.load(os.path.join(ol.GOLDEN, "trained_net.npz"))
    w = NNetWrapper(device="cpu")
    ol.trained_net(w.nnet)
    for planes, P, v in zip(d["planes"], d["P"], d["v"]):
        p2, v2 = w.predict(planes.astype(np.int64))
        np.testing.assert_allclose(p2, P, rtol=1e-5, atol=1e-7)
        np.testing.assert_allclose(v2[0], v, rtol=1e-5, atol=1e-6)
    assert float(d["trained_max_prior"]) > 5 * float(d["init_max_prior"])
    assert float(d["trained_entropy"]) < float(d["init_entropy"]) - 1.0
