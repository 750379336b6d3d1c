"""The small-batch probe forms (tools/small_probes.py, tools/libazg_small_probes.so: the forms that
measured slower than the product's per-layer kernels and left the product library) held to bit-identity
with the product's azg_small.hip kernels: the one-launch forward azg_small_net (round 5) and the f32-MFMA
3x3 layers azg_small_conv_mfma (round 6)."""
import os
import sys

import pytest
import torch

import oracle_lib as ol

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import small_probes as sp  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,depth,A", [(7, 4, 343), (6, 2, 37), (8, 2, 65)])
@pytest.mark.parametrize("trained", [False, True])
def test_small_mfma_bit_identical_to_valu(n, depth, A, trained):
    """The small-batch 3x3 layers on the f32 MFMA (azg_small_conv_mfma) reproduce the VALU
    kernels' P and v bit for bit at 1-4 leaves: the same slices of the same k-ordered fmaf chains
    (v_mfma_f32_16x16x4_f32 is such a chain per output), summed in the same order.  Boards whose
    layers the MFMA path does not cover (8x8 Othello's conv3: 18-step slices) run the VALU kernels
    under either setting; the repeat checks the tickets are left zero between launches."""
    import azg_amd  # noqa: F401
    from azg_amd.nnet import InferenceNet, InflexionNNet
    if trained and n != 7:
        pytest.skip("the trained network is the 7x7 Inflexion one")
    torch.manual_seed(0)
    net = InflexionNNet(n=n, depth=depth, action_size=A).cuda().eval()
    if trained:
        ol.trained_net(net)
    mf, va = sp.ProbeInferenceNet(net, mode="mfma"), InferenceNet(net)
    print("MFMA layers:", mf.mfma_layout)
    if n in (6, 7):
        assert set(mf.mfma_layout) == {2, 3, 4}
    g = torch.Generator(device="cuda").manual_seed(n + 10 * depth)
    for B in (1, 2, 3, 4, 1):
        x = (torch.rand((B, depth, n, n), generator=g, device="cuda") < 0.3).float()
        if depth > 2:
            x[:, 1] *= 1 - x[:, 0]
            x[:, 2] = float(B * 37 % 343)
            x[:, 3] = float(B % 2)
        with torch.no_grad():
            p1, v1 = mf(x)
            p2, v2 = va(x)
        assert torch.equal(p1, p2) and torch.equal(v1, v2), (B, float((p1 - p2).abs().max()))


@pytest.mark.parametrize("n,depth,A,blocks", [(7, 4, 343, 0), (6, 2, 37, 0), (8, 2, 65, 0), (7, 4, 343, 1),
                                              (7, 4, 343, 7), (6, 2, 37, 3)])
@pytest.mark.parametrize("B", [1, 2, 4])
def test_small_fused_forward_bit_identical(n, depth, A, blocks, B):
    """azg_small_net (the whole small-batch forward in one launch, the layers' blocks as items of an
    in-order work queue) gives P, v bit-identical to the per-layer small kernels and within 1e-5 of
    the module, over 40 launches with changing planes (a stale activation read across a layer
    boundary would show as a mismatch); no wait timed out.  blocks: the launch's grid (0 = one per
    CU; 1, 3, 7: far fewer blocks than items, as when other work holds most of the CUs -- the
    queue must not need its blocks co-resident)."""
    import azg_amd  # noqa: F401
    sp.check(sp.lib().azg_small_net_blocks(blocks), "azg_small_net_blocks")
    try:
        _fused_vs_layers(n, depth, A, B)
    finally:
        sp.lib().azg_small_net_blocks(0)


def _fused_vs_layers(n, depth, A, B):
    from azg_amd.nnet import InferenceNet, InflexionNNet
    torch.manual_seed(20 + n)
    net = InflexionNNet(n=n, depth=depth, action_size=A).cuda().eval()
    fused = sp.ProbeInferenceNet(net, conv="miopen", gemm="f32", mode="fused").cuda()
    layers = InferenceNet(net, conv="miopen", gemm="f32").cuda()
    for i in range(40):
        x = (torch.rand(B, depth, n, n, device="cuda") < 0.3).float()
        if depth == 4:
            x[:, 2:] = x[:, 2:, :1, :1]
        with torch.no_grad():
            pf, vf = fused(x)
            pl, vl = layers(x)
            if i % 10 == 0:
                logp, vr = net(x)
                torch.testing.assert_close(pf, torch.exp(logp), rtol=1e-5, atol=1e-7)
                torch.testing.assert_close(vf.reshape(-1), vr.reshape(-1), rtol=1e-5, atol=1e-6)
        assert torch.equal(pf, pl) and torch.equal(vf, vl), i
    fused.check_fused()


def _contend_worker(rank, q):
    """One of two processes driving fused small-batch forwards on the same GPU at once."""
    try:
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
        import azg_amd  # noqa: F401
        from azg_amd.nnet import InferenceNet, InflexionNNet
        torch.manual_seed(31)
        net = InflexionNNet(n=7, depth=4, action_size=343).cuda().eval()
        import small_probes as sp_
        fused = sp_.ProbeInferenceNet(net, conv="miopen", gemm="f32", mode="fused").cuda()
        layers = InferenceNet(net, conv="miopen", gemm="f32").cuda()
        g = torch.Generator(device="cuda").manual_seed(rank)
        xs = [(torch.rand(1, 4, 7, 7, device="cuda", generator=g) < 0.3).float() for _ in range(300)]
        with torch.no_grad():
            outs = [fused(x) for x in xs]  # back to back: the two processes' launches overlap
            torch.cuda.synchronize()
            bad = sum(not (torch.equal(p, pl) and torch.equal(v, vl))
                      for (p, v), (pl, vl) in zip(outs, (layers(x) for x in xs)))
        fused.check_fused()
        q.put((rank, bad, None))
    except Exception as e:  # noqa: BLE001
        q.put((rank, -1, repr(e)))


def test_small_fused_forward_two_processes():
    """Two processes on one GPU launching the fused forward concurrently (each launch's grid is one
    block per CU, so neither can have all of its blocks resident while the other runs): every
    result bit-identical to the per-layer kernels and no wait timed out -- a grid barrier here timed
    out (tests/test_gpu_dist.py's two ranks on one GPU, round 5), the work queue must not."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_contend_worker, args=(r, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict((r, (bad, err)) for r, bad, err in (q.get(timeout=150) for _ in ps))
    for p in ps:
        p.join(timeout=30)
    assert res[0] == (0, None) and res[1] == (0, None), res
