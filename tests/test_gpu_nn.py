"""GPU leaf network: the inference form (BN folded, NHWC, fused bias+ReLU HIP
epilogue) against the reference module on the same planes (f32, 1e-5 rel)."""
import os

import numpy as np
import pytest
import torch

import oracle_lib as ol

pytestmark = pytest.mark.gpu


def test_bias_relu_kernel():
    import azg_amd  # noqa: F401
    from azg_amd.nnet import _bias_relu_
    x = torch.randn(37, 512, 5, 5, device="cuda").contiguous(memory_format=torch.channels_last)
    b = torch.randn(512, device="cuda")
    want = torch.relu(x + b.view(1, -1, 1, 1))
    got = _bias_relu_(x.clone(memory_format=torch.channels_last), b)
    assert torch.equal(got, want)


@pytest.mark.parametrize("conv,gemm", [("miopen", "split"), ("azg", "split"), ("auto", "split"),
                                       ("winograd", "split"), ("winograd", "split_blas"), ("winograd", "f32")])
def test_inference_net_vs_reference_gpu(conv, gemm):
    import azg_amd  # noqa: F401
    from azg_amd.nnet import InferenceNet, InflexionNNet
    d = dict(np.load(ol.os.path.join(ol.GOLDEN, "nnet_golden.npz")))
    torch.manual_seed(0)
    net = InflexionNNet().eval()
    x = torch.from_numpy(d["planes"].astype(np.float32))
    fast = InferenceNet(net.cuda(), conv=conv, gemm=gemm).cuda()
    with torch.no_grad():
        p, v = fast(x.cuda())
    fast.check_range()
    np.testing.assert_allclose(p.cpu().numpy(), d["P"], rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(v.cpu().numpy().ravel(), d["v"], rtol=1e-5, atol=1e-6)


def test_graph_replay_matches_eager():
    import azg_amd  # noqa: F401
    from azg_amd.engine import SelfPlayEngine
    from azg_amd.nnet import InferenceNet, InflexionNNet
    torch.manual_seed(0)
    net = InferenceNet(InflexionNNet().cuda().eval())
    a = SelfPlayEngine(64, sims=8, evaluator=net, max_turns=343)
    b = SelfPlayEngine(64, sims=8, evaluator=net, max_turns=343)
    a.move()
    b.move()
    b.capture_move()
    for _ in range(3):
        a.move()
        b.move()
    ra, rb = a.read_moves(), b.read_moves()
    assert np.array_equal(ra["counts"][:, :4], rb["counts"][:, :4])
    assert np.array_equal(ra["actions"][:, :4], rb["actions"][:, :4])
    assert a.stats()["expansions"] == b.stats()["expansions"]


@pytest.mark.parametrize("B,H,pad", [(1, 7, 1), (37, 7, 1), (300, 7, 0), (129, 5, 0), (64, 8, 1), (64, 6, 0)])
def test_azg_conv3x3_matches_torch(B, H, pad):
    """libazg implicit-GEMM conv (+bias, ReLU) vs torch conv2d on ragged batch sizes."""
    import azg_amd  # noqa: F401
    from azg_amd.nnet import _azg_conv3x3
    torch.manual_seed(1)
    C = N = 512
    w = torch.randn(N, C, 3, 3, device="cuda") * 0.02
    b = torch.randn(N, device="cuda") * 0.1
    wt = w.permute(2, 3, 1, 0).reshape(9 * C, N).contiguous()
    x = torch.relu(torch.randn(B, C, H, H, device="cuda")).contiguous(memory_format=torch.channels_last)
    want = torch.relu(torch.nn.functional.conv2d(x, w, b, padding=pad))
    got = _azg_conv3x3(x, wt, b, pad)
    torch.testing.assert_close(got, want, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4, 5])
@pytest.mark.parametrize("B,H,pad", [(37, 7, 1), (129, 5, 0), (3, 6, 1)])
def test_azg_conv3x3_variants(variant, B, H, pad):
    """Every libazg conv tile variant (incl. the LDS-DMA ring) on ragged pixel counts."""
    import ctypes
    import azg_amd  # noqa: F401
    from azg_amd import _lib
    torch.manual_seed(2)
    C = N = 512
    w = torch.randn(N, C, 3, 3, device="cuda") * 0.02
    b = torch.randn(N, device="cuda") * 0.1
    wt = w.permute(2, 3, 1, 0).reshape(9 * C, N).contiguous()
    x = torch.relu(torch.randn(B, H, H, C, device="cuda"))
    want = torch.relu(torch.nn.functional.conv2d(x.permute(0, 3, 1, 2), w, b, padding=pad)).permute(0, 2, 3, 1)
    Ho = H + 2 * pad - 2
    y = torch.full((B, Ho, Ho, N), float("nan"), device="cuda")
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    _lib.check(_lib.lib().azg_conv3x3_variant(variant, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(wt.data_ptr()),
                                              ctypes.c_void_p(b.data_ptr()), ctypes.c_void_p(y.data_ptr()),
                                              B, H, pad, C, N, s))
    torch.cuda.synchronize()
    torch.testing.assert_close(y, want, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("gemm", ["split", "split_blas", "f32"])
@pytest.mark.parametrize("B,H,pad", [(1, 7, 1), (37, 7, 1), (300, 7, 0), (129, 5, 0), (64, 8, 1), (5, 6, 0),
                                     (3, 4, 1), (7, 9, 1), (2, 11, 0), (3, 3, 1)])
def test_winograd_conv3x3_matches_torch(B, H, pad, gemm):
    """Winograd layer (mixed F(5,3)/F(4,3)/F(3,3)/F(2,3) tiles: every tile-type group;
    libazg transforms + split-fp16 or f32 bmm) vs torch conv2d + bias + ReLU, and against
    an f64 convolution within 2e-5 of the layer's largest pre-activation.  Measured
    (tools/wino_layer_error.py, profiles/r02_wino_layer_error.json): split 3.4-8.4e-6,
    split_blas / f32 GEMMs up to 1.6e-5 (F(5,3)); torch's direct f32 conv 0.3-1e-6."""
    import azg_amd  # noqa: F401
    from azg_amd.nnet import InferenceNet, InflexionNNet
    torch.manual_seed(3)
    net = InflexionNNet(n=max(H, 5)).eval()
    fast = InferenceNet(net, conv="winograd", gemm=gemm).cuda()
    C = N = 512
    w = torch.randn(N, C, 3, 3) * 0.02
    layer = 2
    fast.set_winograd_layer(layer, w.cuda(), H + 2 * pad - 2)
    b = (torch.randn(N) * 0.1).cuda()
    setattr(fast, f"b{layer}", b)
    x = torch.relu(torch.randn(B, C, H, H, device="cuda")).contiguous(memory_format=torch.channels_last)
    want = torch.relu(torch.nn.functional.conv2d(x, w.cuda(), b, padding=pad))
    got = fast._conv_winograd(x, layer, pad)
    fast.check_range()
    torch.testing.assert_close(got, want, rtol=1e-4, atol=1e-4)
    pre64 = torch.nn.functional.conv2d(x.double(), w.cuda().double(), None, padding=pad)
    want64 = torch.relu(pre64 + b.double().view(1, -1, 1, 1))
    assert (got.double() - want64).abs().max().item() <= 2e-5 * pre64.abs().max().item()


@pytest.mark.parametrize("gemm", ["split", "split_blas", "f32"])
def test_winograd_fused_transforms_match_unfused(gemm):
    """The fused front end (conv1 + conv2's input transform) and the fused
    output/next-input transforms (default) vs MIOpen conv1 and separate
    transforms: same math, conv1 summed in another order (1e-5)."""
    import azg_amd  # noqa: F401
    from azg_amd.nnet import InferenceNet, InflexionNNet
    torch.manual_seed(4)
    net = InflexionNNet().cuda().eval()
    a, b = InferenceNet(net, gemm=gemm).cuda(), InferenceNet(net, gemm=gemm).cuda()
    b.fuse_transforms = False
    x = (torch.rand(300, 4, 7, 7, device="cuda") < 0.3).float()
    with torch.no_grad():
        pa, va = a(x)
        pb, vb = b(x)
    torch.testing.assert_close(pa, pb, rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(va, vb, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("gemm", ["split", "split_blas", "f32"])
@pytest.mark.parametrize("n,depth,A", [(7, 4, 343), (6, 2, 37), (8, 2, 65), (5, 4, 175), (9, 2, 82), (9, 4, 567)])
def test_inference_net_board_sizes(n, depth, A, gemm):
    """The inference form (fused front end, fused Winograd transforms; register
    planes for the supported boards, LDS planes otherwise) vs the reference module."""
    import azg_amd  # noqa: F401
    from azg_amd.nnet import InferenceNet, InflexionNNet
    torch.manual_seed(n)
    net = InflexionNNet(n=n, depth=depth, action_size=A).cuda().eval()
    fast = InferenceNet(net, gemm=gemm).cuda()
    x = (torch.rand(160, depth, n, n, device="cuda") < 0.3).float()
    with torch.no_grad():
        p, v = fast(x)
        logp, v_ref = net(x)
    fast.check_range()
    torch.testing.assert_close(p, torch.exp(logp), rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(v.reshape(-1), v_ref.reshape(-1), rtol=1e-5, atol=1e-6)


def test_split_gemm_flags_fp16_overflow():
    """A split-GEMM operand fp16 cannot hold is reported, not silently wrong."""
    import azg_amd  # noqa: F401
    from azg_amd.nnet import InferenceNet, InflexionNNet
    torch.manual_seed(5)
    net = InflexionNNet().cuda().eval()
    fast = InferenceNet(net).cuda()
    x = torch.full((64, 4, 7, 7), 1e6, device="cuda")
    with torch.no_grad():
        fast(x)
    with pytest.raises(FloatingPointError):
        fast.check_range()
    fast.check_range()  # the flag was cleared


def test_split_gemm_error_not_above_f32():
    """The split-fp16 forward's error against an f64 forward of the same inference
    form is no larger than the f32-GEMM forward's (4096 leaves of random planes)."""
    import azg_amd  # noqa: F401
    from azg_amd.nnet import InferenceNet, InflexionNNet
    torch.manual_seed(6)
    net = InflexionNNet().cuda().eval()
    ref = InflexionNNet().cuda().eval().double()
    ref.load_state_dict(net.state_dict())
    x = (torch.rand(1024, 4, 7, 7, device="cuda") < 0.3).float()
    with torch.no_grad():
        logp, v64 = ref(x.double())
        p64 = torch.exp(logp)
        errs = {}
        for gemm in ("split", "split_blas", "f32"):
            p, v = InferenceNet(net, gemm=gemm).cuda()(x)
            errs[gemm] = ((p.double() - p64).abs() / p64).max().item()
    assert errs["split"] < 1e-5 and errs["split_blas"] < 1e-5, errs
    assert errs["split"] <= 1.5 * errs["f32"], errs
    assert errs["split_blas"] <= 1.5 * errs["f32"], errs


def _rescaled(net, layer, factor, nxt):
    """`net` with BatchNorm `layer`'s gamma, beta times `factor` and the next layer's weights
    divided by it: the same function, its activations between the two layers `factor` times smaller."""
    import copy
    out = copy.deepcopy(net)
    with torch.no_grad():
        bn = getattr(out, layer)
        bn.weight.mul_(factor)
        bn.bias.mul_(factor)
        for name in (nxt if isinstance(nxt, tuple) else (nxt,)):
            getattr(out, name).weight.div_(factor)
    return out


def _split_errors(net, x, band=None):
    """Max relative P error and max absolute v error of the split / f32-GEMM forms against an f64
    forward of `net` (band: nnet.ACT_BAND for the call, e.g. (0, inf) = no activation scaling)."""
    import azg_amd.nnet as nn_mod
    ref = type(net)().cuda().eval().double()
    ref.load_state_dict(net.state_dict())
    saved = nn_mod.ACT_BAND
    if band is not None:
        nn_mod.ACT_BAND = band
    try:
        with torch.no_grad():
            logp, v64 = ref(x.double())
            p64 = torch.exp(logp)
            out = {}
            for gemm in ("split", "f32"):
                fast = nn_mod.InferenceNet(net, gemm=gemm).cuda()
                p, v = fast(x)
                fast.check_range()
                out[gemm] = (((p.double() - p64).abs() / p64).max().item(),
                             (v.double().reshape(-1) - v64.reshape(-1)).abs().max().item())
    finally:
        nn_mod.ACT_BAND = saved
    return out


@pytest.mark.parametrize("layer,nxt", [("bn1", "conv2"), ("bn2", "conv3"), ("bn3", "conv4"), ("bn4", "fc1"),
                                       ("fc_bn1", "fc2"), ("fc_bn2", ("fc3", "fc4"))])
def test_split_gemm_error_small_activations(layer, nxt):
    """a split-GEMM operand below 2^-3 has its low half in fp16's subnormals.
    A network whose BatchNorm shrinks one layer's activations by 1e-5 (the next layer's weights
    grown to match: the same function) is evaluated with that layer rescaled by a power of two
    (nnet.act_exponent), and its split forward stays within the f32-GEMM form's error and the
    north_star's 1e-5 of an f64 forward -- 1024 leaves (split-K fc1 and the split FC tail).
    Unscaled (ACT_BAND disabled) the same network's error is printed for comparison (CPU model,
    tools/wino_error_sim.py: P 8.8e-6, v 4.3e-6 at conv3's input)."""
    import azg_amd  # noqa: F401
    from azg_amd.nnet import InflexionNNet
    torch.manual_seed(6)
    net = _rescaled(InflexionNNet().cuda().eval(), layer, 1e-5, nxt).eval()
    x = (torch.rand(1024, 4, 7, 7, device="cuda") < 0.3).float()
    scaled = _split_errors(net, x)
    unscaled = _split_errors(net, x, band=(0.0, float("inf")))
    print(f"{layer} x 1e-5: scaled split P {scaled['split'][0]:.3g} v {scaled['split'][1]:.3g} (f32 GEMMs P "
          f"{scaled['f32'][0]:.3g} v {scaled['f32'][1]:.3g}); unscaled split P {unscaled['split'][0]:.3g} "
          f"v {unscaled['split'][1]:.3g}")
    assert scaled["split"][0] < 1e-5 and scaled["split"][1] < 1e-5, scaled
    assert scaled["split"][0] <= 1.5 * scaled["f32"][0] + 1e-7, scaled
    assert scaled["split"][1] <= 1.5 * scaled["f32"][1] + 1e-7, scaled


def test_split_gemm_error_trained_network():
    """The split forward on the network the reference trains on its own self-play
    (tests/golden/trained_net.npz, make_golden.py trained_net): within the f32-GEMM form's
    error and 1e-5 of an f64 forward, on 1024 leaves of the positions of random playouts and
    their random symmetries plus random planes."""
    import azg_amd  # noqa: F401
    from azg_amd.nnet import InflexionNNet
    net = ol.trained_net(InflexionNNet()).cuda().eval()
    d = np.load(os.path.join(ol.GOLDEN, "trained_net.npz"))
    pos = torch.from_numpy(d["planes"].astype(np.float32)).cuda()
    rnd = (torch.rand(1024 - pos.shape[0], 4, 7, 7, device="cuda") < 0.3).float()
    rnd[:, 2:] = rnd[:, 2:, :1, :1]  # the turn and can_spawn planes are constant
    x = torch.cat([pos, rnd])
    e = _split_errors(net, x)
    print(f"trained network: split P {e['split'][0]:.3g} v {e['split'][1]:.3g}, f32 GEMMs P {e['f32'][0]:.3g} "
          f"v {e['f32'][1]:.3g}")
    assert e["split"][0] < 1e-5 and e["split"][1] < 1e-5, e
    assert e["split"][0] <= 1.5 * e["f32"][0] + 1e-7, e
    assert e["split"][1] <= 1.5 * e["f32"][1] + 1e-7, e


@pytest.mark.parametrize("conv,gemm", [("winograd", "split"), ("winograd", "f32"), ("miopen", "f32")])
@pytest.mark.parametrize("B", [1, 64, 1024])
def test_inference_net_trained_network(conv, gemm, B):
    """The inference forms on the trained network reproduce the reference NNetWrapper's batch-1
    CPU predict on its 64 fixture positions (make_golden.py trained_net) within 1e-5; B leaves
    (the positions tiled): the small-batch kernels at 1, the Winograd forms from 64."""
    import azg_amd  # noqa: F401
    from azg_amd.nnet import InferenceNet, InflexionNNet
    net = ol.trained_net(InflexionNNet()).cuda().eval()
    d = np.load(os.path.join(ol.GOLDEN, "trained_net.npz"))
    x = torch.from_numpy(d["planes"].astype(np.float32)).cuda()
    idx = torch.arange(B, device="cuda") % x.shape[0]
    fast = InferenceNet(net, conv=conv, gemm=gemm).cuda()
    with torch.no_grad():
        p, v = fast(x[idx])
    fast.check_range()
    np.testing.assert_allclose(p.cpu().numpy(), d["P"][idx.cpu().numpy()], rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(v.cpu().numpy().ravel(), d["v"][idx.cpu().numpy()], rtol=1e-5, atol=1e-6)


PROBE_VARIANTS = [1, 2, 3, 5, 7, 8, 11, 12, 19]  # tools/libazg_probes.so only (HISTORY.md 4.1)
probes = pytest.mark.skipif(not os.environ.get("AZG_PROBES"),
                            reason="probe-only GEMM schedules: AZG_PROBES=1 (tools/Makefile builds them)")


@pytest.mark.parametrize("variant", [0, 4, 17, 18] + [pytest.param(v, marks=probes) for v in PROBE_VARIANTS])
@pytest.mark.parametrize("runs,C,K", [([(25, 4096)], 512, 512), ([(3, 300), (5, 37), (2, 513)], 512, 512),
                                      ([(1, 1)], 512, 512), ([(2, 77), (1, 256)], 64, 256),
                                      ([(4, 129)], 128, 768), ([(17, 4000)], 64, 512), ([(11, 3000)], 64, 512),
                                      ([(3, 385), (2, 768), (1, 383)], 64, 512)])
def test_split_gemm_kernel_matches_reference(variant, runs, C, K):
    """libazg azg_split_gemm (hand-written fp16 MFMA, LDS-DMA): M = Ah.Bh + Al.Bh + Ah.Bl
    for every point of every run, against the same products in f64 (ragged row counts,
    the smallest channel counts, every kernel schedule; the last three shapes leave a
    partial last round of the persistent grid, ragged ones included)."""
    _check_split_gemm(variant, runs, C, K)


@pytest.mark.parametrize("runs,C,K", [([(9, 4096)], 512, 512), ([(8, 2048), (8, 4096)], 512, 512),
                                      ([(17, 4000)], 64, 512), ([(49, 256)], 512, 512), ([(25, 256)], 512, 512),
                                      ([(121, 1024)], 64, 512)])
def test_split_gemm_default_schedule_matches_reference(runs, C, K):
    """azg_split_gemm's own schedule: 256-row persistent tiles, or 128-row tiles for short
    launches (the 256-leaf shapes), ragged and multi-run shapes included."""
    _check_split_gemm(None, runs, C, K)


@pytest.mark.parametrize("runs,C,K", [([(121, 4096)], 512, 512), ([(4, 4096)], 1152, 1024),
                                      ([(3, 385), (2, 768), (1, 383)], 64, 512)])
@probes
def test_split_gemm_384_rows_bit_equal_to_256_rows(runs, C, K):
    """Variant 19 (384 x 256 tiles) runs every accumulator's MFMAs in variant 4's order
    (stage by stage, hi.hi, lo.hi, hi.lo): the same bits, so a schedule pick between
    the two never changes the network's outputs."""
    outs = [_run_split_gemm(v, runs, C, K)[2] for v in (4, 19)]
    assert torch.equal(outs[0], outs[1])


def test_split_gemm_grid_cap_bit_equal():
    """azg_set_gemm_blocks caps the persistent grid (fewer CUs, more tiles per block):
    each tile's arithmetic is unchanged, so the results are the uncapped launch's bits;
    a negative cap is rejected."""
    import azg_amd  # noqa: F401
    from azg_amd import _lib
    L = _lib.lib()
    runs = [(3, 385), (2, 768)]
    ref = _run_split_gemm(4, runs, 64, 512)[2]
    try:
        for cap in (1, 7, 8, 100, 200):
            _lib.check(L.azg_set_gemm_blocks(cap))
            assert torch.equal(_run_split_gemm(4, runs, 64, 512)[2], ref), cap
    finally:
        _lib.check(L.azg_set_gemm_blocks(0))
    assert L.azg_set_gemm_blocks(-1) == -1


def test_product_library_has_no_probe_schedules():
    """The probe-only schedules live in tools/libazg_probes.so: the product library
    rejects them (and exports no stamp build)."""
    import ctypes
    import azg_amd  # noqa: F401
    from azg_amd import _lib
    L = _lib.lib()
    assert not hasattr(L, "azg_split_gemm_stamps")
    x = torch.zeros(256 * 1024, dtype=torch.float16, device="cuda")
    m = torch.zeros(256 * 256, device="cuda")
    pts, rows = (ctypes.c_int32 * 1)(1), (ctypes.c_int32 * 1)(256)
    for v in PROBE_VARIANTS:
        assert L.azg_split_gemm_variant(v, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(x.data_ptr()),
                                        ctypes.c_void_p(m.data_ptr()), 1, pts, rows, 512, 256,
                                        ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)) == -1, v


def _run_split_gemm(variant, runs, C, K):
    import ctypes
    import azg_amd  # noqa: F401
    from azg_amd import _lib
    torch.manual_seed(7)
    P = sum(p for p, _ in runs)
    A = torch.cat([torch.randn(p * t, 2 * C, device="cuda").half() for p, t in runs]).contiguous()
    Bt = torch.randn(P, K, 2 * C, device="cuda").half()
    M = torch.full((sum(p * t for p, t in runs) * K,), float("nan"), device="cuda")
    pts = (ctypes.c_int32 * len(runs))(*[p for p, _ in runs])
    rows = (ctypes.c_int32 * len(runs))(*[t for _, t in runs])
    ptrs = (ctypes.c_void_p(A.data_ptr()), ctypes.c_void_p(Bt.data_ptr()), ctypes.c_void_p(M.data_ptr()),
            len(runs), pts, rows, C, K, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    if variant is None:
        _lib.check(_lib.lib().azg_split_gemm(*ptrs))
    elif variant in (0, 4, 17, 18):
        _lib.check(_lib.lib().azg_split_gemm_variant(variant, *ptrs))
    else:
        _lib.check(_lib.probes().azg_split_gemm_variant(variant, *ptrs))
    torch.cuda.synchronize()
    return A, Bt, M


def _check_split_gemm(variant, runs, C, K):
    from azg_amd.nnet import split2_halves
    A, Bt, M = _run_split_gemm(variant, runs, C, K)
    a_row = m_row = pt = 0
    for p, t in runs:
        a = A[a_row:a_row + p * t].view(p, t, 2 * C).double()
        b = Bt[pt:pt + p].double()
        (ah, al), (bh, bl) = split2_halves(a), split2_halves(b)  # 32-channel [hi | lo] blocks
        want = ah @ bh.transpose(1, 2) + al @ bh.transpose(1, 2) + ah @ bl.transpose(1, 2)
        got = M[m_row * K:(m_row + p * t) * K].view(p, t, K).double()
        scale = want.abs().max().item()
        assert (got - want).abs().max().item() <= 2e-6 * scale, (p, t)
        a_row += p * t
        m_row += p * t
        pt += p


@pytest.mark.parametrize("extra", [0, 277])
def test_fc1_split_form_matches_reference(extra):
    """At >= FC1_SPLIT_MIN_BATCH leaves the FC tail runs as split-fp16 GEMMs: fc1 over
    conv4's [hi|lo|hi] output rows (azg_winograd_out_split), fc2 and [fc3 | fc4] over the
    rows azg_fc_act_split writes, P and v from azg_policy_value (fc1 on libazg's split
    GEMM as a split-K GEMM, or on hipBLASLt): against the reference module within the
    north_star's 1e-5, and equal to the f32 FC tail within it."""
    import azg_amd  # noqa: F401
    from azg_amd import nnet as nn_mod
    from azg_amd.nnet import InferenceNet, InflexionNNet
    torch.manual_seed(9)
    net = InflexionNNet().cuda().eval()
    fast = InferenceNet(net).cuda()
    assert fast.fc1_split
    x = (torch.rand(nn_mod.FC1_SPLIT_MIN_BATCH + extra, 4, 7, 7, device="cuda") < 0.3).float()  # ragged tiles too
    assert fast.fc1_kparts == nn_mod.FC1_KPARTS
    assert fast.fc_tail_azg
    with torch.no_grad():
        p, v = fast(x)                  # fc1, fc2, [fc3 | fc4] all as libazg split-K split GEMMs
        logp, v_ref = net(x)
        fast.fc_tail_azg = False
        pa, va = fast(x)                # fc1 on libazg, fc2 and [fc3 | fc4] on hipBLASLt
        fast.fc1_kparts = 0
        pb, vb = fast(x)                # fc1 as the hipBLASLt split GEMM
        fast.fc1_split = False
        p32, v32 = fast(x)              # f32 FC tail
    fast.check_range()
    for pp, vv in ((p, v), (pa, va), (pb, vb)):
        torch.testing.assert_close(pp, torch.exp(logp), rtol=1e-5, atol=1e-7)
        torch.testing.assert_close(vv.reshape(-1), v_ref.reshape(-1), rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(pp, p32, rtol=1e-5, atol=1e-7)


def test_fc_act_split_kernel():
    """azg_fc_act_split against the torch f32 expression relu(b + s sum_p m_p): hi =
    fp16(y), lo = fp16(y - hi), rows [hi | lo | hi]; one part and four split-K parts
    (summed in order); an out-of-range value sets the flag."""
    import ctypes
    from azg_amd import _lib
    B, n, scale = 300, 1024, 2.0 ** -7
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for parts in (1, 4):
        m = torch.randn(parts, B, n, device="cuda") * 300
        b = torch.randn(n, device="cuda")
        out = torch.empty(B, 3 * n, device="cuda", dtype=torch.float16)
        ovf = torch.zeros(1, dtype=torch.int32, device="cuda")

        def run():
            _lib.check(_lib.lib().azg_fc_act_split(ctypes.c_void_p(m.data_ptr()), parts, B * n,
                                                   ctypes.c_void_p(b.data_ptr()), scale,
                                                   ctypes.c_void_p(out.data_ptr()), B, n, 1,
                                                   ctypes.c_void_p(ovf.data_ptr()), st))
        run()
        acc = m[0].clone()
        for p in range(1, parts):
            acc = acc + m[p]
        y = torch.relu(b + scale * acc)
        hi = y.half()
        lo = (y - hi.float()).half()
        assert torch.equal(out[:, :n], hi) and torch.equal(out[:, n:2 * n], lo) and torch.equal(out[:, 2 * n:], hi)
        assert int(ovf.item()) == 0
        m[0, 7, 5] = 1e9
        run()
        assert int(ovf.item()) == 1


@pytest.mark.parametrize("n,out_parts,parts", [(1024, 8, 3), (512, 4, 3), (512, 1, 3), (256, 2, 3), (512, 8, 9),
                                                (512, 8, 16), (256, 4, 20)])
def test_fc_act_split2_layout(n, out_parts, parts):
    """azg_fc_act with AZG_WINO_SPLIT2 output: the same hi / lo values as the [hi | lo | hi]
    form, laid out as out_parts K-parts of 32-channel [hi | lo] blocks (nnet.split2_rows of
    each part), the A operand of the next split-K split GEMM.  Input parts summed in order,
    bit-exact: <= 4 and <= 16 parts (every part's load in flight) and 20 (one at a time)."""
    import ctypes
    from azg_amd import _lib
    from azg_amd.nnet import split2_rows
    B, scale = 257, 2.0 ** -5
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    m = torch.randn(parts, B, n, device="cuda") * 50
    b = torch.randn(n, device="cuda")
    ovf = torch.zeros(1, dtype=torch.int32, device="cuda")
    out = torch.empty(out_parts, B, 2 * n // out_parts, device="cuda", dtype=torch.float16)
    _lib.check(_lib.lib().azg_fc_act(ctypes.c_void_p(m.data_ptr()), parts, B * n, ctypes.c_void_p(b.data_ptr()),
                                     scale, ctypes.c_void_p(out.data_ptr()), B, n, 1, 2, out_parts,
                                     ctypes.c_void_p(ovf.data_ptr()), st))
    acc = m[0].clone()
    for p in range(1, parts):
        acc = acc + m[p]
    y = torch.relu(b + scale * acc)
    hi = y.half()
    lo = (y - hi.float()).half()
    want = split2_rows(hi.reshape(B, out_parts, n // out_parts).transpose(0, 1),
                       lo.reshape(B, out_parts, n // out_parts).transpose(0, 1))
    assert torch.equal(out, want)
    assert int(ovf.item()) == 0
    # a host-memory flag is refused at the boundary (a device atomic to it would fault the GPU)
    host_flag = torch.zeros(1, dtype=torch.int32)
    assert _lib.lib().azg_fc_act(ctypes.c_void_p(m.data_ptr()), parts, B * n, ctypes.c_void_p(b.data_ptr()),
                                 scale, ctypes.c_void_p(out.data_ptr()), B, n, 1, 2, out_parts,
                                 ctypes.c_void_p(host_flag.data_ptr()), st) == -1


@pytest.mark.parametrize("parts,A", [(1, 343), (4, 343), (8, 343), (13, 343), (16, 343), (5, 567)])
def test_policy_value_parts_kernel(parts, A):
    """azg_policy_value_parts: the split-K parts of [fc3 | fc4] summed in order, then softmax / tanh
    (up to 8 parts / up to 16 parts, every part's load in flight; 17 parts refused)."""
    import ctypes
    from azg_amd import _lib
    B, ld, scale = 333, 512 if A < 512 else 640, 0.25
    m = torch.randn(parts, B, ld, device="cuda") * 4
    b = torch.randn(A + 1, device="cuda")
    P = torch.empty(B, A, device="cuda")
    v = torch.empty(B, device="cuda")
    _lib.check(_lib.lib().azg_policy_value_parts(ctypes.c_void_p(m.data_ptr()), parts, B * ld, ld,
                                                 ctypes.c_void_p(b.data_ptr()), scale, ctypes.c_void_p(P.data_ptr()),
                                                 ctypes.c_void_p(v.data_ptr()), B, A,
                                                 ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))
    acc = m[0].clone()
    for p in range(1, parts):
        acc = acc + m[p]
    x = b + scale * acc[:, :A + 1]
    torch.testing.assert_close(P, torch.softmax(x[:, :A], dim=1), rtol=2e-6, atol=1e-8)
    torch.testing.assert_close(v, torch.tanh(x[:, A]), rtol=2e-6, atol=1e-7)
    assert _lib.lib().azg_policy_value_parts(ctypes.c_void_p(m.data_ptr()), 17, B * ld, ld,
                                             ctypes.c_void_p(b.data_ptr()), scale, ctypes.c_void_p(P.data_ptr()),
                                             ctypes.c_void_p(v.data_ptr()), B, A, None) == -1


@pytest.mark.parametrize("A", [343, 65, 36, 512, 567, 1024])
def test_policy_value_kernel(A):
    """azg_policy_value against torch f32 softmax / tanh of the stacked [fc3 | fc4] output."""
    import ctypes
    from azg_amd import _lib
    B, ld, scale = 777, A + 3, 0.5
    m = torch.randn(B, ld, device="cuda") * 8
    b = torch.randn(A + 1, device="cuda")
    P = torch.empty(B, A, device="cuda")
    v = torch.empty(B, 1, device="cuda")
    _lib.check(_lib.lib().azg_policy_value(ctypes.c_void_p(m.data_ptr()), ld, ctypes.c_void_p(b.data_ptr()), scale,
                                           ctypes.c_void_p(P.data_ptr()), ctypes.c_void_p(v.data_ptr()), B, A,
                                           ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))
    logits = b + scale * m[:, :A + 1]
    torch.testing.assert_close(P, torch.softmax(logits[:, :A], dim=1), rtol=2e-6, atol=1e-9)
    torch.testing.assert_close(v, torch.tanh(logits[:, A:]), rtol=2e-6, atol=1e-7)


@pytest.mark.parametrize("kind", ["dense", "mixed", "board6", "board8"])
def test_first_layer_any_planes(kind):
    """winograd_first's conv1 takes per-plane shortcuts (constant planes by border
    class, zero cells skipped); any plane values must give the reference module's
    P, v: dense random floats (no shortcut applies), and a mix of constant, all-zero,
    sparse and dense planes, on 7x7 and on the Othello board sides."""
    import azg_amd  # noqa: F401
    from azg_amd.nnet import InferenceNet, InflexionNNet
    n, depth, A = {"board6": (6, 2, 37), "board8": (8, 2, 65)}.get(kind, (7, 4, 343))
    torch.manual_seed(3)
    net = InflexionNNet(n=n, depth=depth, action_size=A).cuda().eval()
    fast = InferenceNet(net).cuda()
    B = 96
    if kind == "dense":
        x = torch.randn(B, depth, n, n, device="cuda")
    else:
        x = (torch.rand(B, depth, n, n, device="cuda") < 0.2).float()
        x[: B // 3, -1] = 3.5                                             # constant plane
        x[B // 3: 2 * B // 3, 0] = 0.0                                    # all-zero plane
        x[2 * B // 3:, 0] = torch.randn(B - 2 * B // 3, n, n, device="cuda")  # dense plane
        x[5, :, 2, 3] = -0.0                                              # a negative zero
    with torch.no_grad():
        p, v = fast(x)
        logp, v_ref = net(x)
    fast.check_range()
    torch.testing.assert_close(p, torch.exp(logp), rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(v.reshape(-1), v_ref.reshape(-1), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("B,H,pad,cin,cout", [(1, 7, 1, 4, 512), (1, 7, 1, 512, 512), (3, 7, 0, 512, 512),
                                              (1, 5, 0, 512, 512), (1, 7, 0, 512, 512), (2, 8, 1, 2, 512),
                                              (1, 8, 1, 512, 512), (4, 8, 1, 64, 96), (4, 6, 0, 64, 96),
                                              (1, 9, 1, 64, 128), (2, 9, 0, 128, 72), (4, 5, 0, 8, 16),
                                              (1, 3, 1, 20, 2)])
def test_small_conv_matches_torch(B, H, pad, cin, cout):
    """azg_small_conv3x3 (the small path's conv, up to 256 output pixels): a 3x3 conv + bias +
    ReLU against torch in f64, NCHW (scalar loads) and NHWC (float4) inputs, padded and
    unpadded windows, every pixel-tile width (16-256), channel counts that leave K slices of
    unequal length."""
    import ctypes
    import azg_amd  # noqa: F401
    from azg_amd import _lib
    torch.manual_seed(5)
    x = torch.randn(B, cin, H, H, device="cuda")
    w = torch.randn(cout, cin, 3, 3, device="cuda") / (cin * 9) ** 0.5
    b = torch.randn(cout, device="cuda")
    want = torch.relu(torch.nn.functional.conv2d(x.double(), w.double(), b.double(), padding=pad))
    want = want.permute(0, 2, 3, 1).reshape(-1, cout)
    wk = w.contiguous(memory_format=torch.channels_last)
    Ho = H + 2 * pad - 2
    L = _lib.lib()
    work = torch.full((8 * cout * B * Ho * Ho,), float("nan"), device="cuda")
    tickets = torch.zeros(cout // 8 + 1, device="cuda", dtype=torch.int32)
    for layout, split_k in (("nchw", False), ("nhwc", False), ("nhwc", True), ("nhwc", True)):
        if layout == "nchw":
            xin, strides = x.contiguous(), (cin * H * H, H, 1, H * H)
        else:
            xin = x.permute(0, 2, 3, 1).contiguous()
            strides = (H * H * cin, H * cin, cin, 1)
        y = torch.full((B * Ho * Ho, cout), float("nan"), device="cuda")
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        wp = ctypes.c_void_p(work.data_ptr()) if split_k else None
        tp = ctypes.c_void_p(tickets.data_ptr()) if split_k else None
        _lib.check(L.azg_small_conv3x3(ctypes.c_void_p(xin.data_ptr()), *strides, B, H, pad,
                                       ctypes.c_void_p(wk.data_ptr()), cin, cout, ctypes.c_void_p(b.data_ptr()), 1,
                                       ctypes.c_void_p(y.data_ptr()), cout, wp, work.numel() if split_k else 0,
                                       tp, tickets.numel() if split_k else 0, st))
        torch.cuda.synchronize()
        err = ((y.double() - want).abs() / (want.abs() + 1.0)).max().item()
        assert err < 1e-5, (layout, split_k, err)
        assert int(tickets.abs().sum()) == 0  # the split-K form leaves its tickets at zero


@pytest.mark.parametrize("B,K,N,relu,bias", [(1, 4608, 1024, 1, True), (4, 4608, 1024, 1, True),
                                              (1, 1024, 512, 1, True), (3, 1024, 512, 1, True),
                                              (1, 512, 344, 0, False), (2, 512, 66, 0, False),
                                              (1, 8192, 1024, 1, True), (4, 36, 5, 1, True)])
def test_small_fc_matches_torch(B, K, N, relu, bias):
    """azg_small_fc (the small path's FC layers, 1-4 leaves): y = relu?(b + x W^T) against torch
    in f64; row counts not a multiple of the 4-row block, K not a multiple of the 1024-wide
    block stride, no bias (the [fc3 | fc4] GEMM, whose bias the policy/value kernel adds)."""
    import ctypes
    import azg_amd  # noqa: F401
    from azg_amd import _lib
    torch.manual_seed(7)
    x = torch.randn(B, K, device="cuda")
    w = torch.randn(N, K, device="cuda") / K ** 0.5
    b = torch.randn(N, device="cuda") if bias else None
    want = x.double() @ w.double().t() + (b.double() if bias else 0.0)
    if relu:
        want = torch.relu(want)
    y = torch.full((B, N), float("nan"), device="cuda")
    _lib.check(_lib.lib().azg_small_fc(ctypes.c_void_p(x.data_ptr()), K, B, ctypes.c_void_p(w.data_ptr()), K, N,
                                       ctypes.c_void_p(b.data_ptr()) if bias else None, relu,
                                       ctypes.c_void_p(y.data_ptr()), N,
                                       ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))
    torch.cuda.synchronize()
    err = ((y.double() - want).abs() / (want.abs() + 1.0)).max().item()
    assert err < 1e-5, err


@pytest.mark.parametrize("B,depth,n,C", [(1, 4, 7, 512), (4, 4, 7, 512), (2, 2, 6, 512), (3, 2, 8, 512),
                                         (1, 1, 6, 32), (4, 3, 7, 64), (2, 4, 8, 32), (1, 4, 6, 512)])
def test_small_conv12_matches_torch(B, depth, n, C):
    """azg_small_conv12 (conv1 + conv2 in one launch, each split-K block recomputing conv1 for its
    quarter of conv2's input channels): relu(conv2(relu(conv1(planes)))) against torch in f64,
    padded 3x3 convs, 1-4 planes (0/1 and dense), the boards' sides 6..8, the tickets left at zero."""
    import ctypes
    import azg_amd  # noqa: F401
    from azg_amd import _lib
    torch.manual_seed(11)
    x = (torch.rand(B, depth, n, n, device="cuda") < 0.3).float()
    x[:, -1] = torch.randn(B, n, n, device="cuda")
    w1 = torch.randn(C, depth, 3, 3, device="cuda") / (depth * 9) ** 0.5
    w2 = torch.randn(C, C, 3, 3, device="cuda") / (C * 9) ** 0.5
    b1, b2 = torch.randn(C, device="cuda"), torch.randn(C, device="cuda")
    F = torch.nn.functional
    want = torch.relu(F.conv2d(torch.relu(F.conv2d(x.double(), w1.double(), b1.double(), padding=1)),
                               w2.double(), b2.double(), padding=1)).permute(0, 2, 3, 1).reshape(-1, C)
    w1k = w1.contiguous(memory_format=torch.channels_last)
    w2k = w2.contiguous(memory_format=torch.channels_last)
    work = torch.full((8 * C * B * n * n,), float("nan"), device="cuda")
    tickets = torch.zeros(C // 8, device="cuda", dtype=torch.int32)
    V = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    for _ in range(2):
        y = torch.full((B * n * n, C), float("nan"), device="cuda")
        _lib.check(_lib.lib().azg_small_conv12(V(x), B, depth, n, V(w1k), V(b1), V(w2k), V(b2), C, V(y), C, V(work),
                                               work.numel(), V(tickets), tickets.numel(),
                                               ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))
        torch.cuda.synchronize()
        err = ((y.double() - want).abs() / (want.abs() + 1.0)).max().item()
        assert err < 1e-5, err
        assert int(tickets.abs().sum()) == 0


@pytest.mark.parametrize("B,K,A", [(1, 512, 343), (4, 512, 343), (3, 512, 37), (2, 64, 1), (1, 36, 1023)])
def test_small_heads_match_torch(B, K, A):
    """azg_small_heads ([fc3 | fc4] + softmax / tanh in one launch, the heads by the last block
    to finish): P, v against torch in f64 and the logits written out; ticket left at zero."""
    import ctypes
    import azg_amd  # noqa: F401
    from azg_amd import _lib
    torch.manual_seed(13)
    x = torch.randn(B, K, device="cuda")
    w = torch.randn(A + 1, K, device="cuda") / K ** 0.5
    b = torch.randn(A + 1, device="cuda")
    lg = x.double() @ w.double().t()
    P_ref = torch.softmax(lg[:, :A] + b.double()[:A], 1)
    v_ref = torch.tanh(lg[:, A] + b.double()[A])
    logits = torch.full((B, A + 1), float("nan"), device="cuda")
    P = torch.full((B, A), float("nan"), device="cuda")
    v = torch.full((B, 1), float("nan"), device="cuda")
    ticket = torch.zeros(1, device="cuda", dtype=torch.int32)
    V = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    for _ in range(2):
        _lib.check(_lib.lib().azg_small_heads(V(x), K, B, V(w), K, A, V(b), V(logits), V(P), V(v), V(ticket),
                                              ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))
        torch.cuda.synchronize()
        assert ((logits.double() - lg).abs() / (lg.abs() + 1)).max().item() < 1e-5
        torch.testing.assert_close(P.double(), P_ref, rtol=1e-5, atol=1e-7)
        torch.testing.assert_close(v.double().reshape(-1), v_ref, rtol=1e-5, atol=1e-6)
        assert int(ticket.item()) == 0


def test_small_kernels_reject_bad_arguments():
    """Shapes the small kernels do not serve return AZG_ERR_ARG instead of launching."""
    import ctypes
    import azg_amd  # noqa: F401
    from azg_amd import _lib
    L = _lib.lib()
    x = torch.zeros(8 * 8 * 8 * 64, device="cuda")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    P = ctypes.c_void_p(x.data_ptr())
    assert L.azg_small_conv3x3(P, 64 * 64, 64 * 8, 64, 1, 5, 8, 1, P, 64, 64, None, 1, P, 64, None, 0, None, 0,
                               st) == -1  # 5 leaves
    assert L.azg_small_conv3x3(P, 64 * 49, 64 * 7, 64, 1, 1, 7, 1, P, 64, 63, None, 1, P, 64, None, 0, None, 0,
                               st) == -1  # odd Cout
    assert L.azg_small_fc(P, 64, 5, P, 64, 8, None, 1, P, 8, st) == -1  # batch 5
    assert L.azg_small_fc(P, 62, 1, P, 62, 8, None, 1, P, 8, st) == -1  # K % 4
    assert L.azg_small_conv12(P, 1, 5, 7, P, P, P, P, 512, P, 512, P, 1 << 20, P, 64, st) == -1  # depth 5
    assert L.azg_small_conv12(P, 1, 4, 9, P, P, P, P, 512, P, 512, P, 1 << 20, P, 64, st) == -1  # n 9
    assert L.azg_small_conv12(P, 1, 4, 5, P, P, P, P, 512, P, 512, P, 1 << 20, P, 64, st) == -1  # n 5
    assert L.azg_small_conv12(P, 1, 4, 7, P, P, P, P, 520, P, 520, P, 1 << 20, P, 65, st) == -1  # C % 16
    assert L.azg_small_heads(P, 64, 1, P, 64, 1024, P, P, P, P, P, st) == -1  # A > 1023
    assert L.azg_small_heads(P, 64, 5, P, 64, 8, P, P, P, P, P, st) == -1  # batch 5


@pytest.mark.parametrize("n,depth,A,B", [(7, 4, 343, 1), (7, 4, 343, 2), (7, 4, 343, 4), (6, 2, 37, 1),
                                         (6, 2, 37, 4), (8, 2, 65, 1), (8, 2, 65, 3)])
def test_small_forward_matches_reference(n, depth, A, B):
    """Up to SMALL_MAX_B leaves InferenceNet runs on libazg's small-batch kernels (no MIOpen /
    hipBLASLt; the default): P and v within the north_star's 1e-5 of the reference module,
    and of the MIOpen form; per leaf the same bits whatever the batch (batch invariance)."""
    import azg_amd  # noqa: F401
    from azg_amd.nnet import InferenceNet, InflexionNNet
    torch.manual_seed(0)
    net = InflexionNNet(n=n, depth=depth, action_size=A).cuda().eval()
    x = (torch.rand(B, depth, n, n, device="cuda") < 0.3).float()
    if depth > 2:
        x[:, 2] = 17.0
    small = InferenceNet(net)
    lib_form = InferenceNet(net, conv="miopen", small=False)
    assert small.small_path and not lib_form.small_path
    with torch.no_grad():
        p, v = small(x)
        p2, v2 = lib_form(x)
        logp, v_ref = net(x)
    torch.testing.assert_close(p, torch.exp(logp), rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(v.reshape(-1), v_ref.reshape(-1), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(p, p2, rtol=1e-5, atol=1e-7)


def test_split_form_under_expandable_segments():
    """the range flag's device check (azg_ptr.h, hipPointerGetAttributes) must
    accept torch's expandable-segment (VMM) allocations, or the default split evaluator
    would fail with AZG_ERR_ARG under PYTORCH_HIP_ALLOC_CONF=expandable_segments:True."""
    import subprocess
    import sys
    code = (
        "import torch, azg_amd\n"
        "from azg_amd.nnet import InferenceNet, InflexionNNet\n"
        "torch.manual_seed(0)\n"
        "net = InflexionNNet().cuda().eval()\n"
        "x = (torch.rand(256, 4, 7, 7, device='cuda') < 0.3).float()\n"
        "a = InferenceNet(net)\n"
        "b = InferenceNet(net)\n"
        "with torch.no_grad():\n"
        "    for _ in range(2):\n"
        "        pa, va = a(x)\n"
        "        pb, vb = b(x)\n"
        "    ref = torch.exp(net(x)[0])\n"
        "torch.cuda.synchronize()\n"
        "assert torch.equal(pa, pb)\n"
        "assert ((pa - ref).abs() / ref).max().item() < 1e-5\n"
        "print('ok', torch.cuda.memory._get_current_allocator if hasattr(torch.cuda.memory, '_get_current_allocator') else '')\n")
    env = dict(os.environ, PYTORCH_HIP_ALLOC_CONF="expandable_segments:True",
               PYTORCH_CUDA_ALLOC_CONF="expandable_segments:True")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code], env=env, cwd=root, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr


@pytest.mark.parametrize("A,C", [(1024, 64), (343, 6), (343, 10)])
def test_small_path_gate_falls_back(A, C):
    """shapes the small-batch kernels reject (1024 actions: azg_small_heads takes at
    most 1023; 6 or 10 channels: fc1's K = 9 C is not a multiple of 4) are refused by the gate
    instead of raising AZG_ERR_ARG inside it; the 1024-action net then runs the library path at
    one leaf and matches the module.  (C = 2 mod 4 cannot run the library path either: its
    bias / ReLU pass takes float4 rows.)"""
    import azg_amd  # noqa: F401
    from azg_amd.nnet import InferenceNet, InflexionNNet
    torch.manual_seed(8)
    net = InflexionNNet(action_size=A, num_channels=C).cuda().eval()
    fast = InferenceNet(net, conv="miopen", gemm="f32").cuda()
    x = (torch.rand(1, 4, 7, 7, device="cuda") < 0.3).float()
    assert not fast._small_ok(x)
    if C % 4:
        return
    with torch.no_grad():
        p, v = fast(x)
        logp, v_ref = net(x)
    torch.testing.assert_close(p, torch.exp(logp), rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(v.reshape(-1), v_ref.reshape(-1), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("B", [256, 512, 768])
def test_small_fc_tail_matches_reference(B):
    """The FC tail below FC1_SPLIT_MIN_BATCH leaves on libazg only (InferenceNet._fc_split_small:
    fc1 as the transposed split-K GEMM W1 A^T, azg_fc_act_t, then fc2 / [fc3 | fc4] split-K; C2's
    256 leaves; the default since the epilogues load every part in flight) against the reference
    module (1e-5) and the f32 hipBLASLt tail."""
    import azg_amd  # noqa: F401
    from azg_amd.nnet import InferenceNet, InflexionNNet
    torch.manual_seed(13)
    net = InflexionNNet().cuda().eval()
    fast = InferenceNet(net).cuda()
    assert fast.fc_tail_small and hasattr(fast, "fw1_skT")  # the default (nnet.FC_SMALL_TAIL)
    x = (torch.rand(B, 4, 7, 7, device="cuda") < 0.3).float()
    x[:, 2:] = x[:, 2:, :1, :1]
    with torch.no_grad():
        p, v = fast(x)
        fast.check_range()
        logp, v_ref = net(x)
        fast.fc_tail_small = False
        p32, v32 = fast(x)
    torch.testing.assert_close(p, torch.exp(logp), rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(v.reshape(-1), v_ref.reshape(-1), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(p, p32, rtol=1e-5, atol=1e-7)


def test_fc_act_t_kernel():
    """azg_fc_act_t: transposed partial products [parts][n][rows] summed in order, bias, ReLU,
    written as split2 K-parts -- equal to azg_fc_act on the same partials transposed back."""
    import ctypes
    import azg_amd  # noqa: F401
    from azg_amd import _lib
    torch.manual_seed(14)
    parts, n, rows, out_parts = 5, 1024, 256, 16
    m = torch.randn(parts, n, rows, device="cuda")
    bias = torch.randn(n, device="cuda")
    ovf = torch.zeros(1, dtype=torch.int32, device="cuda")
    a = torch.empty((out_parts, rows, 2 * n // out_parts), dtype=torch.float16, device="cuda")
    b = torch.empty_like(a)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    L = _lib.lib()
    _lib.check(L.azg_fc_act_t(ctypes.c_void_p(m.data_ptr()), parts, n * rows, ctypes.c_void_p(bias.data_ptr()), 0.25,
                              ctypes.c_void_p(a.data_ptr()), rows, n, 1, out_parts, ctypes.c_void_p(ovf.data_ptr()), st))
    mt = m.transpose(1, 2).contiguous()
    _lib.check(L.azg_fc_act(ctypes.c_void_p(mt.data_ptr()), parts, n * rows, ctypes.c_void_p(bias.data_ptr()), 0.25,
                            ctypes.c_void_p(b.data_ptr()), rows, n, 1, 2, out_parts, ctypes.c_void_p(ovf.data_ptr()), st))
    torch.cuda.synchronize()
    assert torch.equal(a.view(torch.int16), b.view(torch.int16))
    assert int(ovf.item()) == 0
