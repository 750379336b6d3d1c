"""The trainer's 3x3 convolutions on libazg's Winograd transforms and split-fp16 GEMM.

NNetWrapper.train (inflexion/pytorch/NNet.py:36-76) spends ~80% of a 512-example step in
conv2-4 of InflexionNNet.forward (InflexionNNet.py:39-45) and their autograd, on MIOpen's
f32 implicit GEMMs (profiles/r05_prof_train_probe.md: ~6.6 of 8.2 ms).  `WinogradConv3x3`
computes the same convolution (raw conv weights and bias; the BatchNorm after it stays
torch's, training mode) and its three gradients in the Winograd domain of the inference
form (nnet.InferenceNet) -- F(4,3)+F(3,3) / F(5,3) / F(3,3) tiles, each
transformed point one split-fp16 GEMM (f32-accurate products on the fp16 MFMA):

    forward   V = B^T x B (azg_winograd_in_nhwc), M = V U (azg_split_gemm), y = A^T M A + b
    backward  dM = A dy A^T, dV = dM U^T, dx = sum of B dV B^T over the overlapping tiles,
              dU = V^T dM (both operands transposed), dw = sum_e G_a^T dU_e G_b (azg_wt_dw),
              db = sum dy

(csrc/azg_wino_train.hip).  Operands are scaled by powers of two chosen on the device (U:
max in (512, 1024]; dy: in (16, 32]) and unscaled exactly, so no step waits on the host.
`train_forward` is InflexionNNet.forward with conv2-4 replaced when `applies` holds (a GPU
batch, 512-style channel counts, the 7x7 board's layer sides) and bn1-4 + ReLU on
BatchNormReLU (NHWC, azg_train_bn.hip; BatchNormReLUDP under the data-parallel trainer's
GlobalBatchNorm, its sums all-reduced) and conv1 on Conv1Train (azg_train_conv1.hip); everything
else -- dropout, the FC layers and their BatchNorms, the losses and Adam -- is the reference's
torch code.
"""
import ctypes

import torch
import torch.nn.functional as F

from . import _lib
from .nnet import winograd_groups, winograd_points

SPLIT2 = 2  # azg.h AZG_WINO_SPLIT2


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _stream(dev):
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def _runs(h_out, B):
    """[(points, rows)] of the layer's GEMMs: tile groups with equal tiles per image merged."""
    runs = []
    for _, _, P, n in winograd_groups(h_out):
        if runs and runs[-1][2] == n:
            runs[-1][0] += P
        else:
            runs.append([P, B * n, n])
    return [(P, rows) for P, rows, _ in runs]


# measurement hook (bench.py --learn-iteration): GEMM_HOOK(what, flops) around every split GEMM launch
# of the training convolutions, "start" / "stop" on the launching stream (eager steps only: nothing is
# recorded inside a graph capture)
GEMM_HOOK = None


def _gemm(A, Bt, M, runs, c, k, dev):
    pts = (ctypes.c_int32 * len(runs))(*[P for P, _ in runs])
    rows = (ctypes.c_int32 * len(runs))(*[r for _, r in runs])
    hook = GEMM_HOOK if not torch.cuda.is_current_stream_capturing() else None
    if hook is not None:
        hook("start", 0.0)
    _lib.check(_lib.lib().azg_split_gemm(_p(A), _p(Bt), _p(M), len(runs), pts, rows, c, k, _stream(dev)))
    if hook is not None:  # executed fp16 MFMA FLOPs: 3 products per f32 multiply-add
        hook("stop", 3.0 * 2.0 * sum(P * r for P, r in runs) * c * k)


def applies(x, conv):
    """Whether conv (nn.Conv2d 3x3) on x runs here: a CUDA batch divisible by 64 (the transposed
    operands of dU), channel counts the split GEMM tiles (in % 64, out % 256 and in % 256 for the
    input-gradient GEMM), and a layer the kernels are built for (7x7 -> 7x7, 7 -> 5, 5 -> 3)."""
    if not (x.is_cuda and x.dim() == 4 and x.dtype == torch.float32 and conv.kernel_size == (3, 3)
            and conv.stride == (1, 1) and conv.bias is not None):
        return False
    B, C, H, W = x.shape
    pad = conv.padding[0]
    return (H == W and (H, pad) in ((7, 1), (7, 0), (5, 0)) and B % 64 == 0 and C % 256 == 0
            and conv.out_channels % 256 == 0 and conv.in_channels == C)


class WinogradConv3x3(torch.autograd.Function):
    """y = conv3x3(x, w) + b (no ReLU) and its gradients on libazg's training kernels.
    x: [B, C, H, H] f32 CUDA (any memory format; channels_last avoids a copy), w: [K, C, 3, 3],
    b: [K].  Returns y [B, K, Ho, Ho] in channels_last memory format."""

    @staticmethod
    def forward(ctx, x, w, b, pad):
        L = _lib.lib()
        dev = x.device
        st = _stream(dev)
        B, C, H, _ = x.shape
        K = w.shape[0]
        Ho = H + 2 * pad - 2
        P = winograd_points(Ho)
        runs = _runs(Ho, B)
        rows = sum(p * r for p, r in runs)
        xc = x.contiguous(memory_format=torch.channels_last)
        wc = w.detach().contiguous()
        ovf = _flag(dev)
        V = torch.empty(rows * 2 * C, dtype=torch.float16, device=dev)
        _lib.check(L.azg_winograd_in_nhwc(_p(xc), None, _p(V), B, H, pad, C, SPLIT2, _p(ovf), st))
        uamax = torch.empty(1, dtype=torch.int32, device=dev)
        ut = torch.empty(P * K * 2 * C, dtype=torch.float16, device=dev)
        un = torch.empty(P * C * 2 * K, dtype=torch.float16, device=dev)
        pm = torch.empty(-(-C * K // 256), dtype=torch.float32, device=dev)  # the build's block maxima of |U|
        _lib.check(L.azg_wt_u_build(_p(wc), C, K, Ho, _p(uamax), _p(ut), _p(un), _p(pm), st))
        M = torch.empty(rows * K, dtype=torch.float32, device=dev)
        _gemm(V, ut, M, runs, C, K, dev)
        y = torch.empty((B, K, Ho, Ho), dtype=torch.float32, device=dev, memory_format=torch.channels_last)
        _lib.check(L.azg_wt_out(_p(M), _p(b.detach().contiguous()), _p(y), B, Ho, K, _p(uamax), st))
        ctx.save_for_backward(V, un, uamax)
        ctx.shape = (B, C, H, K, Ho, pad)
        return y

    @staticmethod
    def backward(ctx, dy):
        L = _lib.lib()
        V, un, uamax = ctx.saved_tensors
        ovf = _flag(dy.device)
        B, C, H, K, Ho, pad = ctx.shape
        dev = dy.device
        st = _stream(dev)
        runs = _runs(Ho, B)
        rows = sum(p * r for p, r in runs)
        P = winograd_points(Ho)
        dyc = dy.contiguous(memory_format=torch.channels_last)
        dyamax = torch.empty(1, dtype=torch.int32, device=dev)
        # max |dy| (the dM scale) and db = dy summed over (batch, h, w) in one read of dy
        db = torch.empty(K, dtype=torch.float32, device=dev) if ctx.needs_input_grad[2] else None
        work = torch.empty(2 * 512 * K + 256, dtype=torch.float64, device=dev)
        _lib.check(L.azg_wt_dy_stats(_p(dyc), B * Ho * Ho, K, _p(dyamax), _p(db), _p(work), st))
        dM = torch.empty(rows * 2 * K, dtype=torch.float16, device=dev)
        _lib.check(L.azg_wt_dout(_p(dyc), _p(dM), B, Ho, K, _p(dyamax), _p(ovf), st))
        dx = None
        if ctx.needs_input_grad[0]:
            dV = torch.empty(rows * C, dtype=torch.float32, device=dev)
            _gemm(dM, un, dV, runs, K, C, dev)
            dx = torch.empty((B, C, H, H), dtype=torch.float32, device=dev, memory_format=torch.channels_last)
            _lib.check(L.azg_wt_din(_p(dV), _p(dx), B, H, pad, C, _p(uamax), _p(dyamax), st))
        dw = None
        if ctx.needs_input_grad[1]:
            # dU_e [C][K] = V_e^T dM_e, contracted over the tiles: operands transposed per run
            dU = torch.empty((P, C, K), dtype=torch.float32, device=dev)
            row = pt = 0
            for Pr, T in runs:
                Vt = torch.empty(Pr * C * 2 * T, dtype=torch.float16, device=dev)
                dMt = torch.empty(Pr * K * 2 * T, dtype=torch.float16, device=dev)
                _lib.check(L.azg_wt_split2_transpose(_p(V[row * 2 * C:]), _p(Vt), Pr, T, C, st))
                _lib.check(L.azg_wt_split2_transpose(_p(dM[row * 2 * K:]), _p(dMt), Pr, T, K, st))
                _gemm(Vt, dMt, dU[pt:pt + Pr], [(Pr, C)], T, K, dev)
                row += Pr * T
                pt += Pr
            # dw[k][c][r][s] = sum over the groups of G_a^T dU G_b, the dy scale undone (azg_wt_dw)
            dw = torch.empty((K, C, 3, 3), dtype=torch.float32, device=dev)
            _lib.check(L.azg_wt_dw(_p(dU), C, K, Ho, _p(dyamax), _p(dw), st))
        return dx, dw, db, None


class Conv1Train(torch.autograd.Function):
    """conv1 (InflexionNNet.py:39: 3x3, stride 1, padding 1) on the board planes, forward and the
    weight / bias gradients on libazg (azg_train_conv1.hip), so no training step reaches MIOpen
    (whose conv1 kernels were compiled on a process's first step: 2.2 s, tools/train_first_use.py).
    x: channels-last planes [B, D, n, n] (no gradient), w: [K, D, 3, 3], b: [K].  Returns y
    channels-last."""

    @staticmethod
    def forward(ctx, x, w, b):
        dev = x.device
        B, D, n, _ = x.shape
        K = w.shape[0]
        y = torch.empty((B, K, n, n), dtype=torch.float32, device=dev, memory_format=torch.channels_last)
        _lib.check(_lib.lib().azg_conv1_train_fwd(_p(x), B, D, n, _p(w.detach().contiguous()), _p(b.detach()), K,
                                                  _p(y), _stream(dev)))
        ctx.save_for_backward(x)
        ctx.K = K
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        dev = x.device
        B, D, n, _ = x.shape
        K = ctx.K
        dyc = dy.contiguous(memory_format=torch.channels_last)
        dw = torch.empty((K, D, 3, 3), dtype=torch.float32, device=dev)
        db = torch.empty(K, dtype=torch.float32, device=dev)
        work = torch.empty(64 * K * (9 * D + 1), dtype=torch.float64, device=dev)
        _lib.check(_lib.lib().azg_conv1_train_wgrad(_p(x), _p(dyc), B, D, n, K, _p(dw), _p(db), _p(work),
                                                    _stream(dev)))
        return None, dw, db


def _conv1_ok(conv, x):
    return (type(conv) is torch.nn.Conv2d and conv.kernel_size == (3, 3) and conv.stride == (1, 1)
            and conv.padding == (1, 1) and conv.dilation == (1, 1) and conv.groups == 1 and conv.bias is not None
            and conv.padding_mode == "zeros" and x.is_cuda and x.dtype == torch.float32 and x.dim() == 4
            and not x.requires_grad and x.is_contiguous(memory_format=torch.channels_last)
            and x.shape[1] == conv.in_channels and x.shape[1] <= 8 and x.shape[2] == x.shape[3] <= 8
            and conv.out_channels % 64 == 0 and 0 < x.shape[0] <= 262140)


def conv1_train(conv, x):
    """conv(x) for the first layer: on Conv1Train when its shapes allow, else the module."""
    if _conv1_ok(conv, x):
        return Conv1Train.apply(x, conv.weight, conv.bias)
    return conv(x)


class BatchNormReLU(torch.autograd.Function):
    """relu(bn(x)) for a training-mode nn.BatchNorm2d on channels-last x, forward and backward on
    libazg's NHWC kernels (azg_train_bn.hip: per-channel sums in f64 over fixed row ranges, the
    ReLU fused, the running statistics updated on the device).  MIOpen's channels-last BatchNorm
    kernels ran at ~1.3 TB/s on the trainer's activations (1.36 ms of a 512-example step,
    profiles/r05_prof_train_probe_wino.md).  Returns y channels-last."""

    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, momentum, eps):
        L = _lib.lib()
        dev = x.device
        B, C, H, W = x.shape
        rows = B * H * W
        y = torch.empty_like(x, memory_format=torch.channels_last)
        sv = torch.empty(4 * C, dtype=torch.float32, device=dev)
        work = torch.empty(1026 * C, dtype=torch.float64, device=dev)
        _lib.check(L.azg_bn_relu_fwd(_p(x), rows, C, _p(weight.detach()), _p(bias.detach()), float(eps),
                                     float(momentum), _p(running_mean), _p(running_var), _p(y), _p(sv), _p(work),
                                     _stream(dev)))
        ctx.save_for_backward(x, sv)
        return y

    @staticmethod
    def backward(ctx, dy):
        L = _lib.lib()
        x, sv = ctx.saved_tensors
        dev = x.device
        B, C, H, W = x.shape
        dyc = dy.contiguous(memory_format=torch.channels_last)
        dx = torch.empty_like(x, memory_format=torch.channels_last)
        dg = torch.empty(C, dtype=torch.float32, device=dev)
        db = torch.empty(C, dtype=torch.float32, device=dev)
        co = torch.empty(2 * C, dtype=torch.float32, device=dev)
        work = torch.empty(1026 * C, dtype=torch.float64, device=dev)
        _lib.check(L.azg_bn_relu_bwd(_p(x), _p(dyc), B * H * W, C, _p(sv), _p(dx), _p(dg), _p(db), _p(co), _p(work),
                                     _stream(dev)))
        return dx, dg, db, None, None, None, None


class BatchNormReLUDP(torch.autograd.Function):
    """BatchNormReLU with the statistics of the whole data-parallel batch (ddp.GlobalBatchNorm's
    arithmetic: every rank holds an equal slice): the per-channel f64 sums of this rank's rows are
    SUM-all-reduced before the finish, forward and backward; dgamma / dbeta are this rank's own
    share (the trainer's gradient all-reduce sums them), dx uses the whole batch's sums."""

    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, momentum, eps, group, world):
        import torch.distributed as dist
        from . import ddp
        L = _lib.lib()
        dev = x.device
        B, C, H, W = x.shape
        rows = B * H * W
        work = torch.empty(1024 * C, dtype=torch.float64, device=dev)
        sums = torch.empty(2 * C, dtype=torch.float64, device=dev)
        _lib.check(L.azg_bn_sums(_p(x), rows, C, _p(sums), _p(work), _stream(dev)))
        dist.all_reduce(sums, op=dist.ReduceOp.SUM, group=group)
        ddp._count("bn_allreduce", sums.numel() * 8)
        y = torch.empty_like(x, memory_format=torch.channels_last)
        sv = torch.empty(4 * C, dtype=torch.float32, device=dev)
        _lib.check(L.azg_bn_relu_fwd_from_sums(_p(x), rows, C, _p(sums), rows * world, _p(weight.detach()),
                                               _p(bias.detach()), float(eps), float(momentum), _p(running_mean),
                                               _p(running_var), _p(y), _p(sv), _stream(dev)))
        ctx.save_for_backward(x, sv)
        ctx.group, ctx.world = group, world
        return y

    @staticmethod
    def backward(ctx, dy):
        import torch.distributed as dist
        from . import ddp
        L = _lib.lib()
        x, sv = ctx.saved_tensors
        dev = x.device
        B, C, H, W = x.shape
        rows = B * H * W
        dyc = dy.contiguous(memory_format=torch.channels_last)
        work = torch.empty(1024 * C, dtype=torch.float64, device=dev)
        sums = torch.empty(2 * C, dtype=torch.float64, device=dev)
        _lib.check(L.azg_bn_relu_bwd_sums(_p(x), _p(dyc), rows, C, _p(sv), _p(sums), _p(work), _stream(dev)))
        db, dg = sums[:C].float(), sums[C:].float()  # this rank's share (before the reduction)
        dist.all_reduce(sums, op=dist.ReduceOp.SUM, group=ctx.group)
        ddp._count("bn_allreduce", sums.numel() * 8)
        dx = torch.empty_like(x, memory_format=torch.channels_last)
        co = torch.empty(2 * C, dtype=torch.float32, device=dev)
        _lib.check(L.azg_bn_relu_bwd_from_sums(_p(x), _p(dyc), rows, C, _p(sv), _p(sums), rows * ctx.world, _p(dx),
                                               None, None, _p(co), _stream(dev)))
        return dx, dg, db, None, None, None, None, None, None


def _bn_relu_ok(bn, x):
    return (type(bn) is torch.nn.BatchNorm2d and bn.training and bn.affine and bn.track_running_stats
            and bn.momentum is not None and x.is_cuda and x.dtype == torch.float32 and x.dim() == 4
            and x.is_contiguous(memory_format=torch.channels_last) and x.shape[1] % 4 == 0
            and x.shape[1] <= 1024 and x.numel() // x.shape[1] >= 2)


def bn_relu(bn, x):
    """relu(bn(x)) as InflexionNNet.forward applies it (InflexionNNet.py:39-45): on
    BatchNormReLU for a plain training-mode nn.BatchNorm2d (affine, running statistics, a
    momentum) over channels-last CUDA f32 activations, on BatchNormReLUDP for the data-parallel
    trainer's GlobalBatchNorm around one, else the module and F.relu (eval mode, other layouts)."""
    if _bn_relu_ok(bn, x):
        bn.num_batches_tracked.add_(1)
        return BatchNormReLU.apply(x, bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.momentum, bn.eps)
    inner = getattr(bn, "bn", None)  # ddp.GlobalBatchNorm: the whole data-parallel batch's statistics
    if inner is not None and type(bn).__name__ == "GlobalBatchNorm" and _bn_relu_ok(inner, x):
        inner.num_batches_tracked.add_(1)
        return BatchNormReLUDP.apply(x, inner.weight, inner.bias, inner.running_mean, inner.running_var,
                                     inner.momentum, inner.eps, bn.group, bn.world)
    return F.relu(bn(x))


def applies_net(net, s):
    """Whether train_forward puts conv2-4 of `net` on the training kernels for planes s: a CUDA
    batch of 64k leaves, the 7x7 board's layer sides (pads 1, 1, 0, 0), channel counts % 256.
    Otherwise NNetWrapper trains the module itself, as the reference does (NCHW, MIOpen)."""
    return (s.is_cuda and s.dtype == torch.float32 and s.numel() // (net.depth * net.n * net.n) % 64 == 0
            and net.n == 7 and net.num_channels % 256 == 0
            and [getattr(net, f"conv{i}").padding[0] for i in range(1, 5)] == [1, 1, 0, 0])


def conv3x3(x, conv):
    """conv(x) on the training kernels when `applies`, else the module itself."""
    if applies(x, conv):
        return WinogradConv3x3.apply(x, conv.weight, conv.bias, conv.padding[0])
    return conv(x)


def train_trunk(net, s):
    """InflexionNNet.forward (InflexionNNet.py:39-53) in training up to fc2's dropout, conv2-4 on the
    Winograd kernels (conv3x3): the input of fc3 and fc4."""
    x = s.view(-1, net.depth, net.n, net.n)
    if x.is_cuda:
        x = x.contiguous(memory_format=torch.channels_last)
    x = bn_relu(net.bn1, conv1_train(net.conv1, x))
    for i in range(2, 5):
        x = bn_relu(getattr(net, f"bn{i}"), conv3x3(x, getattr(net, f"conv{i}")))
    x = x.reshape(x.shape[0], -1)
    x = F.dropout(F.relu(net.fc_bn1(net.fc1(x))), p=net.dropout, training=net.training)
    return F.dropout(F.relu(net.fc_bn2(net.fc2(x))), p=net.dropout, training=net.training)


def train_forward(net, s):
    """InflexionNNet.forward (InflexionNNet.py:39-54) in training, conv2-4 on the Winograd
    kernels (conv3x3).  Returns (log_softmax(fc3), tanh(fc4)) as the module does."""
    x = train_trunk(net, s)
    return F.log_softmax(net.fc3(x), dim=1), torch.tanh(net.fc4(x))


class HeadsLoss(torch.autograd.Function):
    """(l_pi, l_v) of the training step (NNet.py:57-61, 96-100: -sum(t_pi * log_softmax(x3)) / B and
    sum((t_v - tanh(z4))^2) / B) and their gradients w.r.t. the fc3 / fc4 outputs on libazg
    (azg_train_loss.hip): 3 launches per step instead of torch's ~16 (log_softmax, tanh, products, sums,
    negation, divisions and their adjoints).  Returns two 0-dim tensors."""

    @staticmethod
    def forward(ctx, x3, z4, tpi, tv):
        B, A = x3.shape
        x3c, z4c, tpc, tvc = x3.contiguous(), z4.contiguous(), tpi.contiguous(), tv.contiguous()
        rows = torch.empty((B, 4), dtype=torch.float32, device=x3.device)
        out = torch.empty(2, dtype=torch.float32, device=x3.device)
        _lib.check(_lib.lib().azg_train_loss_fwd(_p(x3c), A, _p(z4c), z4c.stride(0), _p(tpc), A, _p(tvc), B, A,
                                                 _p(rows), _p(out), _stream(x3.device)))
        ctx.save_for_backward(x3c, z4c, tpc, tvc, rows)
        return out[0], out[1]

    @staticmethod
    def backward(ctx, g_pi, g_v):
        x3, z4, tpi, tv, rows = ctx.saved_tensors
        B, A = x3.shape
        dev = x3.device
        g = torch.stack([g_pi if g_pi is not None else torch.zeros((), device=dev),
                         g_v if g_v is not None else torch.zeros((), device=dev)]).float().contiguous()
        dx3 = torch.empty_like(x3)
        dz4 = torch.empty_like(z4)
        _lib.check(_lib.lib().azg_train_loss_bwd(_p(x3), A, _p(z4), z4.stride(0), _p(tpi), A, _p(tv), _p(rows), B, A,
                                                 _p(g), _p(dx3), A, _p(dz4), dz4.stride(0), _stream(dev)))
        return dx3, dz4, None, None


def train_losses(net, s, tpi, tv):
    """(l_pi, l_v) of a training step: train_trunk, fc3 / fc4, then HeadsLoss."""
    x = train_trunk(net, s)
    return HeadsLoss.apply(net.fc3(x), net.fc4(x), tpi, tv)


def check_range(device=None):
    """Raise FloatingPointError if a split operand of the training convolutions left fp16's
    range since the last call (an activation above 65504, or a non-finite one; the scaled
    gradients cannot: |dM| <= 32 (sum |A|)^2 <= 30752 for these tiles), and clear the flag."""
    for dev, f in list(_FLAGS.items()):
        if device is not None and dev != _key(device):
            continue
        if int(f.item()):
            f.zero_()
            raise FloatingPointError("training convolution operand out of fp16 range")


def take_flag(device):
    """The out-of-range flag of `device`'s training convolutions since the last call (0 / 1),
    cleared (one host synchronisation)."""
    f = _FLAGS.get(_key(device))
    if f is None:
        return 0
    v = int(f.item())
    if v:
        f.zero_()
    return v


_FLAGS = {}
def _key(dev):
    dev = torch.device(dev)
    if dev.type == "cuda" and dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    return dev


def _flag(dev):
    dev = _key(dev)
    f = _FLAGS.get(dev)
    if f is None:
        f = _FLAGS[dev] = torch.zeros(1, dtype=torch.int32, device=dev)
    return f


__all__ = ["BatchNormReLU", "BatchNormReLUDP", "Conv1Train", "WinogradConv3x3", "applies", "applies_net", "bn_relu",
           "check_range", "conv1_train", "conv3x3", "take_flag", "train_forward"]
