"""fc1's input / output gradient under wino_train.train_forward with conv1 on Conv1Train and on the
module (tools/train_grad_error.py found fc1.weight's gradient 4.7e-2 off an f64 run in the first
case, 8.7e-6 in the second, with equal forward outputs)."""
import sys

import torch

sys.path.insert(0, ".")
import azg_amd  # noqa: E402,F401
import azg_amd.wino_train as wt  # noqa: E402
from azg_amd.nnet import InflexionNNet  # noqa: E402


def run(net, x, tp, tv, conv1_custom):
    saved = {}
    orig = wt._conv1_ok
    if not conv1_custom:
        wt._conv1_ok = lambda conv, xx: False
    h1 = net.fc1.register_forward_hook(lambda m, i, o: saved.__setitem__("a", i[0].detach().clone()))
    h2 = net.fc1.register_full_backward_hook(lambda m, gi, go: saved.__setitem__("dy", go[0].detach().clone()))
    h3 = net.fc_bn1.register_full_backward_hook(lambda m, gi, go: saved.__setitem__("dbn", go[0].detach().clone()))
    net.zero_grad()
    pi, v = wt.train_forward(net, x)
    loss = -torch.sum(tp * pi) / x.shape[0] + torch.sum((tv - v.view(-1)) ** 2) / x.shape[0]
    loss.backward()
    for h in (h1, h2, h3):
        h.remove()
    wt._conv1_ok = orig
    saved["gw"] = net.fc1.weight.grad.detach().clone()
    saved["a_strides"] = saved["a"].stride()
    return saved


def main():
    torch.backends.cudnn.deterministic = True
    torch.manual_seed(12)
    net = InflexionNNet(dropout=0.0).cuda().train()
    x = (torch.rand(128, 4, 7, 7, device="cuda") < 0.3).float()
    tp = torch.softmax(torch.randn(128, 343, device="cuda"), 1)
    tv = torch.rand(128, device="cuda") * 2 - 1
    A = run(net, x, tp, tv, True)
    B = run(net, x, tp, tv, False)
    for k in ("a", "dy", "dbn", "gw"):
        d = (A[k].double() - B[k].double()).abs().max().item() / B[k].abs().max().item()
        print(k, f"{d:.3e}", tuple(A[k].shape), A[k].stride(), B[k].stride())
    # the GEMM itself from A's operands, in f64
    gw64 = A["dy"].double().t() @ A["a"].double()
    print("gw(custom conv1) vs f64 of its own operands", (A["gw"].double() - gw64).abs().max().item() / gw64.abs().max().item())
    gw64b = B["dy"].double().t() @ B["a"].double()
    print("gw(module conv1) vs f64 of its own operands", (B["gw"].double() - gw64b).abs().max().item() / gw64b.abs().max().item())


if __name__ == "__main__":
    main()
