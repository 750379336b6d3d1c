"""Where a fresh process's first training call spends its extra seconds (bench.py's learn iteration
measured 14.8 s as a box's first process, 12.3 s as its second): times, in one process, conv1's
training-mode forward + weight gradient on MIOpen (first call, second call), the FC layers on
hipBLASLt, and two short train_examples calls."""
import json
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
import azg_amd  # noqa: E402,F401
from azg_amd.examples import ExampleSet  # noqa: E402
from azg_amd.inflexion import InflexionGame  # noqa: E402
from azg_amd.nnet import NNetWrapper  # noqa: E402


def timed(fn):
    torch.cuda.synchronize()
    t = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    return time.perf_counter() - t


def main():
    dev = torch.device("cuda")
    out = {}
    x = torch.rand(512, 4, 7, 7, device=dev).contiguous(memory_format=torch.channels_last)
    w = torch.randn(512, 4, 3, 3, device=dev, requires_grad=True)
    b = torch.zeros(512, device=dev, requires_grad=True)

    def conv1():
        y = F.conv2d(x, w, b, padding=1)
        y.sum().backward()
    out["conv1_first_s"] = timed(conv1)
    out["conv1_second_s"] = timed(conv1)
    a = torch.randn(512, 4608, device=dev, requires_grad=True)
    lw = torch.randn(1024, 4608, device=dev, requires_grad=True)

    def fc():
        F.linear(a, lw).sum().backward()
    out["fc1_first_s"] = timed(fc)
    out["fc1_second_s"] = timed(fc)
    bn = torch.nn.BatchNorm1d(1024).to(dev).train()
    z = torch.randn(512, 1024, device=dev, requires_grad=True)

    def bn1d():
        bn(z).sum().backward()
    out["bn1d_first_s"] = timed(bn1d)
    out["bn1d_second_s"] = timed(bn1d)

    def heads():
        q = torch.randn(512, 343, device=dev, requires_grad=True)
        (torch.log_softmax(q, 1).sum() + torch.tanh(q).sum() + torch.nn.functional.dropout(q, 0.3).sum()).backward()
    out["heads_first_s"] = timed(heads)
    out["heads_second_s"] = timed(heads)
    p = [torch.randn(1000, device=dev, requires_grad=True) for _ in range(4)]
    for t in p:
        t.grad = torch.randn_like(t)
    opt = torch.optim.Adam(p, lr=1e-3, capturable=True)
    out["adam_first_s"] = timed(opt.step)
    out["adam_second_s"] = timed(opt.step)
    gen = torch.Generator().manual_seed(3)
    E = 512 * 8
    ex = ExampleSet((torch.rand((E, 4, 7, 7), generator=gen) < 0.3).float().to(dev),
                    torch.softmax(torch.randn((E, 343), generator=gen), 1).to(dev),
                    (torch.randint(0, 2, (E,), generator=gen).float() * 2 - 1).to(dev))
    w0 = NNetWrapper(InflexionGame(7), dict(epochs=1), device="cuda")
    out["train_examples_first_s"] = timed(lambda: w0.train_examples(ex))
    out["train_examples_second_s"] = timed(lambda: w0.train_examples(ex))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
