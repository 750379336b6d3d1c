"""Which training kernel carries conv3.weight's gradient error (tests/test_gpu_wino_train.py::
test_train_forward_matches_module measures 1.3e-2 of max |grad| against an f64 module run): the
same batch through wino_train.train_forward with each Winograd layer in turn put back on the library
(MIOpen f32), and conv1 on Conv1Train or the module; errors of the conv / BatchNorm gradients
against f64."""
import json
import sys

import torch

sys.path.insert(0, ".")
import azg_amd  # noqa: E402,F401
import azg_amd.wino_train as wt  # noqa: E402
from azg_amd.nnet import InflexionNNet  # noqa: E402

KEYS = ["conv1.weight", "conv2.weight", "conv3.weight", "conv4.weight", "bn1.bias", "bn2.bias", "bn3.bias",
        "bn4.bias", "fc1.weight"]


OUTS = {}


def grads(net, x, tp, tv, fwd):
    net.zero_grad()
    pi, v = fwd(x)
    OUTS["last"] = (pi.detach().double(), v.detach().double())
    loss = -torch.sum(tp.to(pi.dtype) * pi) / x.shape[0] + torch.sum((tv.to(v.dtype) - v.view(-1)) ** 2) / x.shape[0]
    loss.backward()
    return {k: p.grad.detach().double().clone() for k, p in net.named_parameters()}


def main():
    torch.backends.cudnn.deterministic = True
    torch.manual_seed(12)
    net = InflexionNNet(dropout=0.0).cuda().train()
    ref = InflexionNNet(dropout=0.0).cuda().train()
    ref.load_state_dict(net.state_dict())
    ref.double()
    x = (torch.rand(128, 4, 7, 7, device="cuda") < 0.3).float()
    tp = torch.softmax(torch.randn(128, 343, device="cuda"), 1)
    tv = torch.rand(128, device="cuda") * 2 - 1
    g64 = grads(ref, x.double(), tp, tv, ref)
    p64, v64 = OUTS["last"]
    orig_applies, orig_c1 = wt.applies, wt._conv1_ok
    out = {}
    layers = {"conv2": (7, 1), "conv3": (7, 0), "conv4": (5, 0)}
    variants = [("conv1_module", None, False), ("all_winograd", None, True)]
    variants += [(f"{n}_library", hp, True) for n, hp in layers.items()]
    variants += [("conv1_module_again", None, False), ("all_winograd_again", None, True)]
    xc = x.contiguous(memory_format=torch.channels_last)
    y1 = wt.Conv1Train.apply(xc, net.conv1.weight, net.conv1.bias)
    y2 = net.conv1(x)
    y3 = ref.conv1(x.double())
    out_c1 = {"conv1train_vs_f64": float((y1.double() - y3).abs().max() / y3.abs().max()),
              "module_vs_f64": float((y2.double() - y3).abs().max() / y3.abs().max())}
    print("conv1_forward", json.dumps(out_c1))
    for name, off, c1 in variants:
        wt.applies = (lambda xx, conv, off=off: orig_applies(xx, conv) and (off is None or (xx.shape[2], conv.padding[0]) != off))
        wt._conv1_ok = orig_c1 if c1 else (lambda conv, xx: False)
        sd = net.state_dict()
        for m in (net.bn1, net.bn2, net.bn3, net.bn4, net.fc_bn1, net.fc_bn2):
            m.reset_running_stats()
        net.load_state_dict(sd)
        g = grads(net, x, tp, tv, lambda s: wt.train_forward(net, s))
        out[name] = {k: float((g[k] - g64[k]).abs().max() / g64[k].abs().max()) for k in KEYS}
        pi, v = OUTS["last"]
        out[name]["pi"] = float((pi.exp() - p64.exp()).abs().max())
        out[name]["v"] = float((v - v64).abs().max())
    wt.applies, wt._conv1_ok = orig_applies, orig_c1
    g = grads(net, x, tp, tv, net)
    out["module_f32"] = {k: float((g[k] - g64[k]).abs().max() / g64[k].abs().max()) for k in KEYS}
    for k, v in out.items():
        print(k, json.dumps({a: f"{b:.2e}" for a, b in v.items()}))


if __name__ == "__main__":
    main()
