"""GPU probe: one Winograd layer's error against an f64 convolution, next to the error of
torch's own f32 convolution (MIOpen) of the same inputs, per output side and GEMM form.
Two input distributions: the layer test's (relu(randn), w ~ 0.02 randn) and the network's
own (random-init InflexionNNet activations).  Prints one JSON line per case.

    python tools/wino_layer_error.py > gpurun_out/wino_layer_error.json
"""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import azg_amd  # noqa: F401
    from azg_amd.nnet import InferenceNet, InflexionNNet, winograd_seq
    torch.manual_seed(3)
    C = N = 512
    for H, pad, B in ((7, 1, 256), (7, 0, 256), (5, 0, 256), (8, 1, 128), (8, 0, 128), (6, 0, 128)):
        h_out = H + 2 * pad - 2
        net = InflexionNNet(n=max(H, 5)).eval()
        w = (torch.randn(N, C, 3, 3) * 0.02).cuda()
        b = (torch.randn(N) * 0.1).cuda()
        x = torch.relu(torch.randn(B, C, H, H, device="cuda")).contiguous(memory_format=torch.channels_last)
        pre64 = F.conv2d(x.double(), w.double(), None, padding=pad)
        want64 = torch.relu(pre64 + b.double().view(1, -1, 1, 1))
        scale = pre64.abs().max().item()
        row = {"h_out": h_out, "tiles": winograd_seq(h_out)}
        with torch.no_grad():
            direct = torch.relu(F.conv2d(x, w, b, padding=pad))
            row["torch_f32_conv"] = (direct.double() - want64).abs().max().item() / scale
            for gemm in ("split", "split_blas", "f32"):
                fast = InferenceNet(net, conv="winograd", gemm=gemm).cuda()
                fast.set_winograd_layer(2, w, h_out)
                fast.b2 = b
                got = fast._conv_winograd(x, 2, pad)
                fast.check_range()
                row[gemm] = (got.double() - want64).abs().max().item() / scale
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
