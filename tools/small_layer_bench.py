"""Per-layer time of azg_small_conv3x3 / azg_small_fc (and the fused conv12 / heads kernels, and
the whole small-path forward) at one leaf (C1's batch) on the 7x7 Inflexion network's
shapes, against torch's conv2d / linear (MIOpen / hipBLASLt, + bias + ReLU) on the same
inputs; medians of round-robin rounds.  Prints one JSON line per layer."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import azg_amd  # noqa: E402,F401
from azg_amd import _lib  # noqa: E402

B = int(os.environ.get("AZG_SL_B", "1"))
LAYERS = [("conv1", 7, 1, 4, 512, "nchw"), ("conv2", 7, 1, 512, 512, "nhwc"), ("conv3", 7, 0, 512, 512, "nhwc"),
          ("conv4", 5, 0, 512, 512, "nhwc"), ("fc1", 1, 0, 4608, 1024, "row"), ("fc2", 1, 0, 1024, 512, "row"),
          ("fc34", 1, 0, 512, 344, "row")]


def timeit(fn, reps=50):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    L = _lib.lib()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for name, H, pad, cin, cout, layout in LAYERS:
        taps = 9 if H > 1 else 1
        x = torch.randn(B, cin, H, H, device="cuda")
        w = torch.randn(cout, cin, 3, 3, device="cuda") if taps == 9 else torch.randn(cout, cin, device="cuda")
        b = torch.randn(cout, device="cuda")
        wk = w.contiguous(memory_format=torch.channels_last) if taps == 9 else w.contiguous()
        if layout == "nchw":
            xin, strides = x.contiguous(), (cin * H * H, H, 1, H * H)
        else:
            xin = x.permute(0, 2, 3, 1).contiguous()
            strides = (H * H * cin, H * cin, cin, 1)
        Ho = H + 2 * pad - 2 if taps == 9 else 1
        y = torch.empty((B * Ho * Ho, cout), device="cuda")
        work = torch.empty(8 * cout * B * Ho * Ho, device="cuda")
        tickets = torch.zeros(cout // 8, device="cuda", dtype=torch.int32)

        def azg(sk=True):
            if taps == 9:
                _lib.check(L.azg_small_conv3x3(ctypes.c_void_p(xin.data_ptr()), *strides, B, H, pad,
                                               ctypes.c_void_p(wk.data_ptr()), cin, cout,
                                               ctypes.c_void_p(b.data_ptr()), 1, ctypes.c_void_p(y.data_ptr()), cout,
                                               ctypes.c_void_p(work.data_ptr()) if sk else None,
                                               work.numel() if sk else 0,
                                               ctypes.c_void_p(tickets.data_ptr()) if sk else None,
                                               tickets.numel() if sk else 0, st))
            else:
                _lib.check(L.azg_small_fc(ctypes.c_void_p(xin.data_ptr()), cin, B, ctypes.c_void_p(wk.data_ptr()),
                                          cin, cout, ctypes.c_void_p(b.data_ptr()), 1,
                                          ctypes.c_void_p(y.data_ptr()), cout, st))

        if taps == 9:
            xcl = x.contiguous(memory_format=torch.channels_last)

            def lib():
                torch.relu_(torch.nn.functional.conv2d(xcl, wk, b, padding=pad))
        else:
            xr = x.reshape(B, cin)

            def lib():
                torch.relu_(torch.addmm(b, xr, w.t()))
        arms = [("azg", azg), ("lib", lib)]
        if taps == 9:  # the one-block-per-2-channels form (no split-K combine)
            arms.append(("azg_nosk", lambda: azg(False)))
        import small_probes as sp
        from small_probes import pack_small_mfma, small_mfma_layout
        lay = small_mfma_layout(H, pad, cin, cout, False) if taps == 9 and layout == "nhwc" else None
        if lay is not None:  # the f32-MFMA form (azg_small_mfma.hip), bit-identical to "azg"
            wm = pack_small_mfma(wk, *lay)
            rows = B * Ho * Ho
            tiles = -(-rows // 16) * (cout // 16)
            mwork = torch.empty(tiles * 256 * max(lay[0], lay[1]), device="cuda")
            mtk = torch.zeros(tiles, device="cuda", dtype=torch.int32)
            y2 = torch.empty_like(y)

            def mfma():
                sp.check(sp.lib().azg_small_conv_mfma(ctypes.c_void_p(xin.data_ptr()), *strides[:3], B, H, pad,
                                                 ctypes.c_void_p(wm.data_ptr()), cin, cout,
                                                 ctypes.c_void_p(b.data_ptr()), 1, ctypes.c_void_p(y2.data_ptr()),
                                                 cout, ctypes.c_void_p(mwork.data_ptr()), mwork.numel(),
                                                 ctypes.c_void_p(mtk.data_ptr()), mtk.numel(), None, None, 0, st),
                         "azg_small_conv_mfma")
            arms.append(("azg_mfma", mfma))
        for _, f in arms:
            for _ in range(5):
                f()
        ts = {k: [] for k, _ in arms}
        for r in range(7):
            for k, f in (arms if r % 2 == 0 else arms[::-1]):
                ts[k].append(timeit(f))
        out = {"layer": name, "B": B, "azg_us": sorted(ts["azg"])[3], "torch_us": sorted(ts["lib"])[3]}
        if "azg_nosk" in ts:
            out["azg_nosk_us"] = sorted(ts["azg_nosk"])[3]
        if "azg_mfma" in ts:
            out["azg_mfma_us"] = sorted(ts["azg_mfma"])[3]
            out["mfma_equal"] = bool(torch.equal(y, y2))
        print(json.dumps(out), flush=True)
    fused(L, st)


def fused(L, st):
    """conv1+conv2 (azg_small_conv12), [fc3|fc4]+heads (azg_small_heads), and the whole small-path
    forward (InferenceNet at B leaves) against the library form (MIOpen / hipBLASLt)."""
    from azg_amd.nnet import InferenceNet, InflexionNNet
    V = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    C, n, depth = 512, 7, 4
    planes = (torch.rand(B, depth, n, n, device="cuda") < 0.3).float()
    w1 = torch.randn(C, depth, 3, 3, device="cuda").contiguous(memory_format=torch.channels_last)
    w2 = torch.randn(C, C, 3, 3, device="cuda").contiguous(memory_format=torch.channels_last)
    b1, b2 = torch.randn(C, device="cuda"), torch.randn(C, device="cuda")
    y = torch.empty(B * n * n, C, device="cuda")
    work = torch.empty(8 * C * B * n * n, device="cuda")
    tickets = torch.zeros(C // 8 + 1, device="cuda", dtype=torch.int32)
    x = torch.randn(B, 512, device="cuda")
    w34, b34 = torch.randn(344, 512, device="cuda"), torch.randn(344, device="cuda")
    lg, P, v = torch.empty(B, 344, device="cuda"), torch.empty(B, 343, device="cuda"), torch.empty(B, device="cuda")
    tk = ctypes.c_void_p(tickets.data_ptr() + 4 * (C // 8))

    def conv12():
        _lib.check(L.azg_small_conv12(V(planes), B, depth, n, V(w1), V(b1), V(w2), V(b2), C, V(y), C, V(work),
                                      work.numel(), V(tickets), C // 8, st))

    import small_probes as sp
    from small_probes import pack_small_mfma, small_mfma_layout
    lay = small_mfma_layout(n, 1, C, C, True)
    wm = pack_small_mfma(w2, *lay)
    tiles = -(-B * n * n // 16) * (C // 16)
    mwork = torch.empty(tiles * 256 * max(lay[0], lay[1]), device="cuda")
    mtk = torch.zeros(tiles, device="cuda", dtype=torch.int32)
    y2 = torch.empty_like(y)

    def conv12_mfma():
        sp.check(sp.lib().azg_small_conv_mfma(V(planes), depth * n * n, 0, 0, B, n, 1, V(wm), C, C, V(b2), 1, V(y2),
                                              C, V(mwork), mwork.numel(), V(mtk), mtk.numel(), V(w1), V(b1), depth,
                                              st), "azg_small_conv_mfma")

    def heads():
        _lib.check(L.azg_small_heads(V(x), 512, B, V(w34), 512, 343, V(b34), V(lg), V(P), V(v), tk, st))
    torch.manual_seed(0)
    net = InflexionNNet().cuda().eval()
    small, lib_form = sp.ProbeInferenceNet(net, mode="mfma"), InferenceNet(net, conv="miopen", small=False)
    valu = InferenceNet(net)
    s = (torch.rand(B, depth, n, n, device="cuda") < 0.3).float()

    def fwd_small():
        small(s)

    def fwd_small_valu():
        valu(s)

    def fwd_lib():
        lib_form(s)
    with torch.no_grad():
        for name, f in (("conv12", conv12), ("conv12_mfma", conv12_mfma), ("heads", heads),
                        ("forward_small", fwd_small), ("forward_small_valu", fwd_small_valu),
                        ("forward_library", fwd_lib)):
            for _ in range(5):
                f()
            t = sorted(timeit(f) for _ in range(7))[3]
            row = {"layer": name, "B": B, "azg_us": t}
            if name == "conv12_mfma":
                row["mfma_equal"] = bool(torch.equal(y, y2))
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
