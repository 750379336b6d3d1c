"""The small-batch forms that measured slower than the product's per-layer VALU kernels, kept as probes
(tools/libazg_small_probes.so, declared in tools/azg_small_probes.h; the product never loads them):

  * the one-launch forward (azg_small_net, round 5): the per-layer kernels' block bodies as the items of
    one in-order work queue -- 125-130 us per one-leaf forward against 65-69 us (cross-XCD activation
    reads and per-item queue atomics cost more than the five kernel boundaries they replace);
  * the f32-MFMA 3x3 layers (azg_small_conv_mfma, round 6): the same slices of the same fmaf chains as
    the VALU kernels (v_mfma_f32_16x16x4_f32 is a k-ordered fmaf chain per output), so bit-identical,
    spread over 256-512 blocks -- conv12 26.5 vs 19.2 us, conv3 16.9 vs 18.0, conv4 17.2 vs 9.3
    (profiles/r06_small_layer_bench.json).

ProbeInferenceNet(net, ..., mode="fused" | "mfma") is an InferenceNet whose small-batch forward takes
one of them; tests/test_gpu_small_probes.py holds both to bit-identity with the product's kernels.
"""
import ctypes
import functools
import os
import subprocess

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
PATH = os.path.join(HERE, "libazg_small_probes.so")
_VP, _I32, _I64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
_L = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE, "libazg_small_probes.so"])
    return PATH


def lib():
    global _L
    if _L is None:
        if not os.path.exists(PATH):
            build()
        L = ctypes.CDLL(PATH)
        for name, args in (
                ("azg_small_net", [_VP, _I32, _I32, _I32, _I32, _I32, _I32, _I32, _VP, _VP, _I64, _VP, _VP, _VP, _I64,
                                   _VP, _I32, _VP, _VP, _VP]),
                ("azg_small_net_blocks", [_I32]),
                ("azg_small_mfma_layout", [_I32, _I32, _I32, _I32, _I32, _VP]),
                ("azg_small_conv_mfma", [_VP, _I64, _I32, _I32, _I32, _I32, _I32, _VP, _I32, _I32, _VP, _I32, _VP,
                                         _I32, _VP, _I64, _VP, _I32, _VP, _VP, _I32, _VP])):
            fn = getattr(L, name)
            fn.restype = ctypes.c_int
            fn.argtypes = args
        _L = L
    return _L


def check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what}: error {rc}")


def small_mfma_layout(H, pad, cin, cout, conv12):
    """(KG, KSL, per) of azg_small_mfma_layout: the K-parts, slices per part and float4 steps per
    slice azg_small.hip's VALU kernels use for this layer (mirrored here so the weights can be
    packed without a library call), or None where azg_small_conv_mfma does not run (ragged slices,
    slice lengths other than the boards' 36 / 9 float4 steps)."""
    ho = H + 2 * pad - 2
    n = ho * ho
    if ho <= 0 or n > 256 or cout % 16:
        return None
    pxl = next(p for p in (16, 32, 64, 128, 256) if n <= p)
    kg = 4 if conv12 else (8 if n > 16 and cin % 32 == 0 and cout % 8 == 0 else 1)
    if cin % (4 * kg):
        return None
    ksl, ks = 512 // pxl, 9 * (cin // kg) // 4
    per = -(-ks // ksl)
    if per * ksl != ks or per not in (9, 36):
        return None
    return kg, ksl, per


def pack_small_mfma(w, kg, ksl, per):
    """A conv weight [Cout][Cin][3][3] (any memory format) -> azg_small_conv_mfma's operand
    [KG][Cout][KSL][4][TP]: part q, channel co, slice s, slot j, step t holds the weight of
    k = 4 (s per + t) + j of the part's tap-major K (k = tap * Cq + ci), t padded to TP = 4 ceil(per / 4)."""
    cout, cin = w.shape[:2]
    cq = cin // kg
    wt = w.permute(0, 2, 3, 1).reshape(cout, 9, kg, cq).permute(2, 0, 1, 3).reshape(kg, cout, 9 * cq)
    wt = wt.reshape(kg, cout, ksl, per, 4).permute(0, 1, 2, 4, 3)
    tp = -(-per // 4) * 4
    out = torch.zeros((kg, cout, ksl, 4, tp), dtype=w.dtype, device=w.device)
    out[..., :per] = wt
    return out.contiguous()


@functools.lru_cache(maxsize=None)
def _probe_class():
    import azg_amd  # noqa: F401
    from azg_amd.nnet import SMALL_MAX_B, InferenceNet

    class ProbeInferenceNet(InferenceNet):
        """InferenceNet whose small-batch forward runs a probe form: mode "fused" (azg_small_net) or
        "mfma" (azg_small_conv_mfma for conv1 + conv2, conv3, conv4; the FC layers as the product's)."""

        def __init__(self, net, *args, mode="fused", **kw):
            super().__init__(net, *args, **kw)
            self.mode = mode
            self.mfma_layout = {}
            if mode == "mfma" and net.depth <= 4 and 6 <= net.n <= 8 and self.pads[:2] == [1, 1]:
                c, h, lays = self.w1.shape[0], net.n, {}
                for i in (2, 3, 4):
                    pad = self.pads[i - 1]
                    lays[i] = small_mfma_layout(h, pad, c, c, conv12=i == 2)
                    h = h + 2 * pad - 2
                if all(lay is not None for lay in lays.values()):  # all three or none: else the VALU kernels
                    self.mfma_layout = lays
                    for i, lay in lays.items():
                        self.register_buffer(f"wm{i}", pack_small_mfma(getattr(self, f"w{i}"), *lay))

        def _convs_small(self, planes, B, dev, st, work, tickets):
            if self.mode != "mfma" or not self.mfma_layout:
                return super()._convs_small(planes, B, dev, st, work, tickets)
            L = lib()
            n, C = self.n, self.w1.shape[0]
            tiles = -(-B * n * n // 16) * (C // 16)
            need = tiles * 256 * max(max(kg, ksl) for kg, ksl, _ in self.mfma_layout.values())
            if getattr(self, "_mfma_work", None) is None or self._mfma_work.numel() < need \
                    or self._mfma_work.device != dev:
                self._mfma_work = torch.empty(need, device=dev, dtype=torch.float32)
                self._mfma_tickets = torch.zeros(tiles, device=dev, dtype=torch.int32)
            work, tickets = self._mfma_work, self._mfma_tickets
            wp, tp = ctypes.c_void_p(work.data_ptr()), ctypes.c_void_p(tickets.data_ptr())
            x, H = planes, n
            for i in (2, 3, 4):
                pad = self.pads[i - 1]
                Ho = H + 2 * pad - 2
                y = torch.empty((B * Ho * Ho, C), device=dev, dtype=torch.float32)
                if i == 2:  # x: the NCHW leaf planes, conv1 computed in the kernel
                    args = (ctypes.c_void_p(planes.data_ptr()), self.depth * n * n, 0, 0)
                    c1 = (ctypes.c_void_p(self.w1.data_ptr()), ctypes.c_void_p(self.b1.data_ptr()), self.depth)
                else:
                    args = (ctypes.c_void_p(x.data_ptr()), H * H * C, H * C, C)
                    c1 = (None, None, 0)
                check(L.azg_small_conv_mfma(*args, B, H, pad, ctypes.c_void_p(getattr(self, f"wm{i}").data_ptr()),
                                            C, C, ctypes.c_void_p(getattr(self, f"b{i}").data_ptr()), 1,
                                            ctypes.c_void_p(y.data_ptr()), C, wp, work.numel(), tp, tickets.numel(),
                                            *c1, st), "azg_small_conv_mfma")
                x, H = y, Ho
            return x, H

        def _forward_small(self, planes):
            if self.mode != "fused":
                return super()._forward_small(planes)
            planes = planes.contiguous()
            B, n, C, A = planes.shape[0], self.n, self.w1.shape[0], self.fw3.shape[0]
            if not (self.depth <= 4 and 6 <= n <= 8 and C % 16 == 0 and self.pads == [1, 1, 0, 0]
                    and B <= SMALL_MAX_B):
                raise ValueError("azg_small_net takes the boards' nets (pads 1, 1, 0, 0) at <= 4 leaves")
            dev = planes.device
            st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
            n1, n2 = self.fw1.shape[0], self.fw2.shape[0]
            need_w = 8 * C * SMALL_MAX_B * n * n
            if getattr(self, "_fused_acts", None) is None or self._fused_acts.device != dev:
                self._fused_work = torch.empty(need_w, device=dev, dtype=torch.float32)
                self._fused_tickets = torch.zeros(max(C // 8, 1) + 1, device=dev, dtype=torch.int32)
                need = SMALL_MAX_B * (n * n * C + (n - 2) ** 2 * C + (n - 4) ** 2 * C + n1 + n2 + A + 1)
                self._fused_acts = torch.empty(need, device=dev, dtype=torch.float32)
                # [0:8] the work queue's counters (zero, and left zero by every launch), [8] error flag
                self._fused_bar = torch.zeros(16, device=dev, dtype=torch.int32)
                ptrs = [self.w1, self.b1, self.w2, self.b2, self.w3, self.b3, self.w4, self.b4, self.fw1, self.fb1,
                        self.fw2, self.fb2, self.fw34, self.fb34]
                self._fused_ptrs = (ctypes.c_void_p * 14)(*[t.data_ptr() for t in ptrs])
            p = torch.empty((B, A), device=dev, dtype=torch.float32)
            v = torch.empty((B, 1), device=dev, dtype=torch.float32)
            bar = self._fused_bar
            check(lib().azg_small_net(
                ctypes.c_void_p(planes.data_ptr()), B, self.depth, n, C, A, n1, n2, self._fused_ptrs,
                ctypes.c_void_p(self._fused_acts.data_ptr()), self._fused_acts.numel(), ctypes.c_void_p(p.data_ptr()),
                ctypes.c_void_p(v.data_ptr()), ctypes.c_void_p(self._fused_work.data_ptr()),
                self._fused_work.numel(), ctypes.c_void_p(self._fused_tickets.data_ptr()),
                self._fused_tickets.numel(), ctypes.c_void_p(bar.data_ptr()), ctypes.c_void_p(bar.data_ptr() + 32),
                st), "azg_small_net")
            return p, v

        def check_range(self):
            self.check_fused()
            super().check_range()

        def check_fused(self):
            """Raise if a wait of the fused forward gave up (a layer's items never all finished: the
            results of that launch are void), and reset its work queue."""
            bar = getattr(self, "_fused_bar", None)
            if bar is not None and int(bar[8].item()) != 0:
                bar.zero_()
                raise RuntimeError("azg_small_net: a layer wait timed out")

    return ProbeInferenceNet


def ProbeInferenceNet(net, *args, mode="fused", **kw):
    return _probe_class()(net, *args, mode=mode, **kw)
