"""The trainer's optimizer: torch.optim.Adam (NNet.py:37, `optim.Adam(self.nnet.parameters())`) as
one libazg launch per step (csrc/azg_adam.hip, azg_adam_step).

torch's capturable foreach Adam -- the form the graph-replayed GPU trainer needs -- issues ~20
multi-tensor kernels and ~54 per-parameter scalar kernels per step (~470 us of a 3.0 ms
512-example step, profiles/r06_prof_train_probe.md).  `FusedAdam` keeps m and v in two flat
device buffers and updates every parameter in one kernel with the same f32 arithmetic (the
capturable foreach form's order of operations; the step count lives on the device, so a captured
step replays correctly).  Interface: the subset of torch.optim.Optimizer the trainers use --
`step()`, `zero_grad(set_to_none)` -- plus `step(grads=...)` for gradients that are not in
`.grad` (the data-parallel trainer's all-reduced flat buffer, ddp.py)."""
import ctypes

import torch

from . import _lib

MAX_SEG = 48  # azg.h AZG_ADAM_MAX_SEG


class FusedAdam:
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8):
        self.params = [p for p in params if p.requires_grad]
        if not self.params:
            raise ValueError("FusedAdam: no parameters")
        if len(self.params) > MAX_SEG:
            raise ValueError(f"FusedAdam: {len(self.params)} parameter tensors (at most {MAX_SEG})")
        dev = self.params[0].device
        for p in self.params:
            if p.device != dev or p.dtype != torch.float32 or not p.is_contiguous():
                raise ValueError("FusedAdam: contiguous f32 parameters on one HIP device")
        if dev.type != "cuda":
            raise _lib.AzgError("FusedAdam runs on a HIP device (no CPU fallback)")
        self.device = dev
        self.lr, self.betas, self.eps = float(lr), (float(betas[0]), float(betas[1])), float(eps)
        n = len(self.params)
        counts = [p.numel() for p in self.params]
        total = sum((c + 3) // 4 * 4 for c in counts)
        self.m = torch.zeros(total, dtype=torch.float32, device=dev)
        self.v = torch.zeros(total, dtype=torch.float32, device=dev)
        self.step_count = torch.zeros(1, dtype=torch.float32, device=dev)
        self._n = n
        self._p = (ctypes.c_void_p * n)(*[p.data_ptr() for p in self.params])
        self._g = (ctypes.c_void_p * n)()
        self._counts = (ctypes.c_int64 * n)(*counts)

    def zero_grad(self, set_to_none=True):
        if set_to_none:
            for p in self.params:
                p.grad = None
            return
        grads = [p.grad for p in self.params if p.grad is not None]
        if grads:
            torch._foreach_zero_(grads)  # one multi-tensor launch, not one per parameter

    def step(self, grads=None):
        """One Adam step of every parameter (gradients: `grads` in parameter order, else each
        parameter's .grad).  torch's global optimizer pre / post step hooks
        (torch.optim.optimizer.register_optimizer_step_pre_hook / _post_hook) run around it."""
        from torch.optim import optimizer as _topt
        for hook in list(getattr(_topt, "_global_optimizer_pre_hooks", {}).values()):
            hook(self, (), {})
        self._step(grads)
        for hook in list(getattr(_topt, "_global_optimizer_post_hooks", {}).values()):
            hook(self, (), {})

    def _step(self, grads):
        gs = grads if grads is not None else [p.grad for p in self.params]
        if len(gs) != self._n:
            raise ValueError(f"FusedAdam.step: {len(gs)} gradients for {self._n} parameters")
        keep = []
        for i, (p, g) in enumerate(zip(self.params, gs)):
            if g is None:
                raise RuntimeError("FusedAdam.step: a parameter has no gradient (every parameter is updated "
                                   "each step, as the trainer's network needs)")
            if g.shape != p.shape or g.dtype != torch.float32 or g.device != self.device:
                raise ValueError(f"FusedAdam.step: gradient {i} does not match its parameter")
            if not g.is_contiguous():
                g = g.contiguous()
            keep.append(g)
            self._g[i] = g.data_ptr()
            if p.data_ptr() != self._p[i]:  # a parameter re-bound (load_state_dict keeps storage)
                self._p[i] = p.data_ptr()
        stream = ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        _lib.check(_lib.lib().azg_adam_step(self._n, self._p, self._g, self._counts,
                                            ctypes.c_void_p(self.m.data_ptr()), ctypes.c_void_p(self.v.data_ptr()),
                                            ctypes.c_void_p(self.step_count.data_ptr()), self.lr, self.betas[0],
                                            self.betas[1], self.eps, stream))
        del keep


__all__ = ["FusedAdam"]
