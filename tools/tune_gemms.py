"""Tune the trainer's library GEMMs once with torch's TunableOp and write the results next to the package
(nnet.TUNABLEOP_RESULTS), which NNetWrapper.train_examples then reads instead of tuning at run time
(NNetWrapper._tuned_gemms).  The shapes: the FC layers at the reference's 512-example batch and at the
data-parallel trainer's 256 / 128 / 64-example slices (2 / 4 / 8 ranks).  TunableOp's own validators
(torch, ROCm, hipBLASLt / rocBLAS versions, the GPU) head the file; a process whose validators differ
rejects it and tunes for itself.

    python tools/tune_gemms.py
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import azg_amd  # noqa: E402,F401
from azg_amd import nnet  # noqa: E402
from azg_amd.examples import ExampleSet  # noqa: E402
from azg_amd.inflexion import InflexionGame  # noqa: E402


def main():
    tun = torch.cuda.tunable
    if os.path.exists(nnet.TUNABLEOP_RESULTS):
        os.remove(nnet.TUNABLEOP_RESULTS)
    tun.set_filename(nnet.TUNABLEOP_RESULTS)  # TunableOp writes it when the process ends
    tun.enable(True)
    tun.tuning_enable(True)
    g = torch.Generator().manual_seed(0)
    for bs in (512, 256, 128, 64):
        torch.manual_seed(0)
        w = nnet.NNetWrapper(InflexionGame(7), dict(epochs=1, batch_size=bs, tunable_gemm="tune"), device="cuda")
        E = bs * 6
        ex = ExampleSet((torch.rand((E, 4, 7, 7), generator=g) < 0.3).float().cuda(),
                        torch.softmax(torch.randn((E, 343), generator=g), 1).cuda(),
                        (torch.randint(0, 2, (E,), generator=g).float() * 2 - 1).cuda())
        np.random.seed(0)
        w.train_examples(ex)
        torch.cuda.synchronize()
        print(f"batch {bs}: {len(tun.get_results())} results", flush=True)
    print("validators:", tun.get_validators(), flush=True)
    for r in tun.get_results():
        print("result:", r, flush=True)


if __name__ == "__main__":
    main()
