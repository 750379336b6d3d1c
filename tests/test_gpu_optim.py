"""optim.FusedAdam (libazg azg_adam_step, one launch per step) against torch.optim.Adam's capturable
foreach form (the trainer's optimizer until round 6; NNet.py:37's Adam on the GPU) on the
InflexionNNet's own parameter shapes: the same f32 arithmetic in the same order, so the updates
agree to a few ulps over many steps, eagerly and replayed from a captured HIP graph."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _net_params(seed=0):
    import azg_amd  # noqa: F401
    from azg_amd.nnet import InflexionNNet
    torch.manual_seed(seed)
    return [p.detach().cuda().clone().requires_grad_(True) for p in InflexionNNet().parameters()]


def _grads(params, k):
    g = torch.Generator(device="cuda").manual_seed(100 + k)
    # gradient scales from 1e-9 to 1e1 (|g| ~ eps included) and exact zeros
    out = []
    for i, p in enumerate(params):
        x = torch.randn(p.shape, generator=g, device="cuda") * 10.0 ** (i % 11 - 9)
        x[..., ::7] = 0.0
        out.append(x)
    return out


def test_fused_adam_matches_torch_capturable_adam():
    """12 steps on the network's parameter shapes, gradients from 1e-9 to 1e1 and exact zeros: the
    fused step's error against an f64 Adam on the same gradients is at most torch's own (x2, and
    a few f32 ulps where torch is exact), per tensor."""
    from azg_amd.optim import FusedAdam
    pa, pb = _net_params(), _net_params()
    p64 = [p.detach().double().clone() for p in pa]
    m64 = [torch.zeros_like(p) for p in p64]
    v64 = [torch.zeros_like(p) for p in p64]
    ta = torch.optim.Adam(pa, capturable=True)
    fb = FusedAdam(pb)
    for k in range(12):
        for i, (p, q, g) in enumerate(zip(pa, pb, _grads(pa, k))):
            p.grad = g.clone()
            q.grad = g.clone()
            g64 = g.double()
            m64[i].mul_(0.9).add_(0.1 * g64)
            v64[i].mul_(0.999).add_(0.001 * g64 * g64)
            bc1, bc2 = 1 - 0.9 ** (k + 1), 1 - 0.999 ** (k + 1)
            p64[i].sub_(1e-3 / bc1 * m64[i] / (v64[i].sqrt() / bc2 ** 0.5 + 1e-8))
        ta.step()
        fb.step()
    torch.cuda.synchronize()
    assert float(fb.step_count) == 12.0
    rows = []
    for p, q, r in zip(pa, pb, p64):
        e_torch = float((p.detach().double() - r).abs().max())
        e_fused = float((q.detach().double() - r).abs().max())
        ulp = 4 * torch.finfo(torch.float32).eps * float(r.abs().max())
        rows.append((tuple(p.shape), e_torch, e_fused))
        assert e_fused <= 2 * e_torch + ulp, (tuple(p.shape), e_torch, e_fused)
    print("max |p - p_f64| (torch, fused):", [(s, f"{a:.2e}", f"{b:.2e}") for s, a, b in rows])


def test_fused_adam_graph_replay_equals_eager():
    from azg_amd.optim import FusedAdam
    pa, pb = _net_params(1), _net_params(1)
    fa, fb = FusedAdam(pa), FusedAdam(pb)
    gbuf = [torch.zeros_like(p) for p in pb]
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):  # warm-up step on a side stream before capture
        fb.step(grads=gbuf)
    torch.cuda.current_stream().wait_stream(side)
    fa.step(grads=[torch.zeros_like(p) for p in pa])
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        fb.step(grads=gbuf)
    for k in range(6):
        gs = _grads(pa, k)
        fa.step(grads=gs)
        for b, g in zip(gbuf, gs):
            b.copy_(g)
        graph.replay()
    torch.cuda.synchronize()
    assert float(fa.step_count) == float(fb.step_count) == 7.0
    for p, q in zip(pa, pb):
        assert torch.equal(p.detach(), q.detach())
    assert torch.equal(fa.m, fb.m) and torch.equal(fa.v, fb.v)


def test_fused_adam_refuses_missing_gradient():
    from azg_amd.optim import FusedAdam
    ps = _net_params()
    f = FusedAdam(ps)
    with pytest.raises(RuntimeError):
        f.step()
