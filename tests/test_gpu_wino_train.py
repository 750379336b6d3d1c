"""The trainer's Winograd convolutions (azg_amd/wino_train.py, csrc/azg_wino_train.hip): conv2-4
of InflexionNNet forward and backward on the Winograd transforms and split-fp16 GEMMs, against
an f64 torch convolution and its autograd (the reference trainer's MIOpen f32 convolutions sit
within ~1e-6 of it)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("H,pad", [(7, 1), (7, 0), (5, 0)])
@pytest.mark.parametrize("B", [64, 512])
def test_winograd_conv_forward_backward(H, pad, B):
    """y, dx, dw, db within 2e-5 of each quantity's largest magnitude (f64 reference); the
    layer shapes of conv2 (7x7 pad 1), conv3 (7 -> 5) and conv4 (5 -> 3) at 512 channels."""
    import azg_amd  # noqa: F401
    from azg_amd.wino_train import WinogradConv3x3, check_range
    torch.manual_seed(11)
    C = K = 512
    x = torch.relu(torch.randn(B, C, H, H, device="cuda")).contiguous(memory_format=torch.channels_last)
    w = torch.randn(K, C, 3, 3, device="cuda") * 0.02
    b = torch.randn(K, device="cuda") * 0.1
    Ho = H + 2 * pad - 2
    dy = torch.randn(B, K, Ho, Ho, device="cuda") * 1e-4  # gradient-sized: far below fp16's normal range
    x1, w1, b1 = (t.clone().requires_grad_() for t in (x, w, b))
    y = WinogradConv3x3.apply(x1, w1, b1, pad)
    y.backward(dy)
    check_range()
    x2, w2, b2 = (t.double().clone().requires_grad_() for t in (x, w, b))
    y2 = torch.nn.functional.conv2d(x2, w2, b2, padding=pad)
    y2.backward(dy.double())
    for name, got, want in (("y", y, y2), ("dx", x1.grad, x2.grad), ("dw", w1.grad, w2.grad),
                            ("db", b1.grad, b2.grad)):
        err = (got.double() - want).abs().max().item() / want.abs().max().item()
        print(f"H {H} pad {pad} B {B}: {name} max error {err:.3g} of max |{name}|")
        assert err < 2e-5, (name, err)


def test_train_forward_matches_module():
    """wino_train.train_forward (conv2-4 on the training kernels) gives the module's training-mode
    outputs and parameter gradients within the f32 tolerance (BatchNorm in training mode, dropout 0)."""
    import azg_amd  # noqa: F401
    from azg_amd.nnet import InflexionNNet
    from azg_amd.wino_train import train_forward
    torch.manual_seed(12)
    net = InflexionNNet(dropout=0.0).cuda().train()
    ref = InflexionNNet(dropout=0.0).cuda().train()
    ref.load_state_dict(net.state_dict())
    x = (torch.rand(128, 4, 7, 7, device="cuda") < 0.3).float()
    tp = torch.softmax(torch.randn(128, 343, device="cuda"), 1)
    tv = torch.rand(128, device="cuda") * 2 - 1
    outs = []
    for m, fwd in ((net, lambda s: train_forward(net, s)), (ref, ref)):
        pi, v = fwd(x)
        loss = -torch.sum(tp * pi) / 128 + torch.sum((tv - v.view(-1)) ** 2) / 128
        loss.backward()
        outs.append((pi.detach(), v.detach(), {k: p.grad.detach().clone() for k, p in m.named_parameters()}))
    (p1, v1, g1), (p2, v2, g2) = outs
    torch.testing.assert_close(p1, p2, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(v1, v2, rtol=1e-4, atol=1e-5)
    for k in g1:
        err = (g1[k] - g2[k]).abs().max().item() / max(g2[k].abs().max().item(), 1e-30)
        # the conv / fc biases ahead of a BatchNorm have a zero gradient up to rounding
        if k.endswith("bias") and k.split(".")[0] in ("conv1", "conv2", "conv3", "conv4", "fc1", "fc2"):
            continue
        assert err < 1e-3, (k, err)
    for name in ("bn2", "bn3", "bn4"):  # running statistics of the training-mode BatchNorm
        np.testing.assert_allclose(getattr(net, name).running_var.cpu().numpy(),
                                   getattr(ref, name).running_var.cpu().numpy(), rtol=1e-4)
