"""Trainer throughput probe: NNetWrapper.train_examples (512 channels, batch 512, Adam)
in memory-format, cudnn.benchmark, Adam and train_dtype variants, on synthetic examples.

    python tools/train_probe.py > gpurun_out/train_probe.json
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import azg_amd  # noqa: E402,F401
from azg_amd.examples import ExampleSet  # noqa: E402
from azg_amd.inflexion import InflexionGame  # noqa: E402
from azg_amd.nnet import NNetWrapper  # noqa: E402


def run(label, channels_last=False, benchmark=False, batches=30, dtype="f32", fused=False, conv="winograd",
        graph_steps=None, **more):
    torch.backends.cudnn.benchmark = benchmark
    torch.manual_seed(0)
    extra = dict(more) if graph_steps is None else {"train_graph_steps": graph_steps, **more}
    w = NNetWrapper(InflexionGame(7), dict(epochs=1, batch_size=512, fused_adam=fused, train_dtype=dtype,
                                           train_conv=conv, **extra), device="cuda")
    if channels_last:
        w.nnet.to(memory_format=torch.channels_last)
    E = 512 * batches
    g = torch.Generator(device="cpu").manual_seed(1)
    planes = (torch.rand((E, 4, 7, 7), generator=g) < 0.3).float().cuda()
    if channels_last:
        planes = planes.contiguous(memory_format=torch.channels_last)
    exs = ExampleSet(planes, torch.softmax(torch.randn((E, 343), generator=g), 1).cuda(),
                     (torch.randint(0, 2, (E,), generator=g).float() * 2 - 1).cuda())
    np.random.seed(0)
    w.train_examples(ExampleSet(exs.planes[:2048], exs.pis[:2048], exs.vs[:2048]))  # warm up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    losses = w.train_examples(exs)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    row = {"form": label, "examples_per_s": E / dt, "TFLOP_per_s": E * 3 * 404.3e6 / dt / 1e12,
           "final_losses": losses[-1].tolist()}
    print(json.dumps(row), flush=True)


if __name__ == "__main__":
    if sys.argv[1:2] == ["f32"]:  # the default trainer alone (e.g. under rocprofv3: kernel time vs wall)
        run("nchw", batches=int(sys.argv[2]) if len(sys.argv) > 2 else 30)
        sys.exit(0)
    if sys.argv[1:2] == ["ab"]:  # one trainer option on / off, alternating: ab <option>
        for _ in range(3):
            for on in (False, True):
                run(f"{sys.argv[2]}={on}", batches=96, **{sys.argv[2]: on})
        sys.exit(0)
    if sys.argv[1:2] == ["tunable"]:  # the FC layers' hipBLASLt GEMMs with torch's TunableOp, alternating
        import tempfile
        for rep in range(2):
            for on in (False, True):
                torch.cuda.tunable.enable(on)
                if on:
                    torch.cuda.tunable.set_filename(os.path.join(tempfile.gettempdir(), "azg_tunableop.csv"))
                    torch.cuda.tunable.set_max_tuning_duration(30)
                run(f"tunableop={on}", batches=96)
        sys.exit(0)
    if sys.argv[1:2] == ["gsteps"]:  # training steps per captured graph, alternating
        for _ in range(2):
            for gsn in (1, 2, 4, 8):
                run(f"graph_steps={gsn}", batches=96, graph_steps=gsn)
        sys.exit(0)
    if sys.argv[1:] == ["conv"]:  # the Winograd training convolutions against the library ones, alternating
        for _ in range(3):
            run("winograd")
            run("library", conv="library")
        sys.exit(0)
    run("nchw")
    run("nchw+benchmark", benchmark=True)
    run("channels_last", channels_last=True)
    run("channels_last+benchmark", channels_last=True, benchmark=True)
    run("nchw+fused_adam", fused=True)
    run("nchw+bf16_autocast", dtype="bf16")
    run("nchw+bf16_autocast+fused_adam", dtype="bf16", fused=True)
