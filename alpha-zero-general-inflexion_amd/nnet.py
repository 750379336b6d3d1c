"""Leaf evaluator: the reference policy/value network on PyTorch-ROCm.

`InflexionNNet` has the reference architecture and parameter names
(inflexion/pytorch/InflexionNNet.py:12-54) so that `{'state_dict': ...}`
checkpoints written by NNetWrapper.save_checkpoint (NNet.py:102-111) load
unchanged, and modules are created in the same order so that
`torch.manual_seed(s)` gives the same random-init weights.

`NNetWrapper` mirrors the reference wrapper surface (NNet.py:27-120):
`predict(planes) -> (P f32[A], v f32[1])` batch-1 as the reference does,
`predict_batch(planes[B,4,n,n]) -> (P [B,A], v [B])` for the engine,
`save_checkpoint` / `load_checkpoint` with the same file format.  Training
(`train`, `train_examples`) runs the reference's loop (batches, losses, Adam):
on the CPU with the reference's arithmetic (bit-identical), on the GPU with
conv2-4 in the Winograd domain and bn1-4 + ReLU on libazg's kernels
(wino_train.py), each step after the third replayed from a captured HIP graph.
"""
import contextlib
import os

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

DEFAULT_ARGS = dict(lr=0.001, dropout=0.3, epochs=10, batch_size=512, num_channels=512,
                    # trainer options beyond the reference (NNet.py:36-76 is f32 + foreach Adam):
                    # fused_adam = one-kernel Adam (+1.5% examples/s; rounds differently where
                    # |grad| ~ eps), train_dtype "bf16" = autocast forward/backward (2.5x
                    # examples/s); both opt-in, not the reference's arithmetic
                    # (profiles/r01_train_probe.json)
                    fused_adam=False, train_dtype="f32",
                    # conv2-4 of the GPU training step: "winograd" (libazg's Winograd transforms and
                    # split-fp16 GEMMs, forward and backward, wino_train.py) or "library" (torch /
                    # MIOpen as the reference).  The CPU trainer is always the reference's.
                    train_conv="winograd")
WINOGRAD_MIN_BATCH = 64  # below this many leaves the Winograd path is slower (C1: 1 game)
# up to SMALL_MAX_B leaves: the whole forward on libazg's small-batch kernels (azg_small.hip: one
# launch per layer, no library) instead of MIOpen / hipBLASLt
SMALL_PATH = True
SMALL_MAX_B = 4
# (the one-launch small-batch forward and the f32-MFMA small-batch 3x3 layers measured slower than the
# per-layer VALU kernels below; they live in the probe library, tools/small_probes.py)
# from this many leaves the FC tail runs fc1 as the 4-part split-K GEMM (FC1_KPARTS); below it (C2's 256)
# as the transposed small-batch form, FC1T_KPARTS / FCS_KPARTS2 / 3 (InferenceNet.fc_tail_small, the
# default; the f32 hipBLASLt tail only when fc_tail_small is off)
FC1_SPLIT_MIN_BATCH = 1024
# NNetWrapper.train_examples on the GPU: steps run eagerly before the step is captured as a HIP graph
_GRAPH_EAGER_STEPS = 3
# training steps per captured HIP graph (args["train_graph_steps"] overrides)
TRAIN_GRAPH_STEPS = 1
# the trainer's FC GEMMs tuned once on an MI355X by torch's TunableOp (tools/tune_gemms.py): read at the
# start of train_examples so that no process spends its first call tuning (NNetWrapper._tuned_gemms)
TUNABLEOP_RESULTS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tunableop_results.csv")
FC1_KPARTS = 4  # split-K parts of fc1 on libazg's split GEMM (4608 = 4 x 1152 for the 7x7 board)
# split-K parts of fc2 (1024 -> 512) and [fc3 | fc4] (512 -> 344, padded to 512 columns) when the whole
# FC tail runs on libazg's split GEMM (InferenceNet.fc_tail_azg): 4 x 256 and 2 x 256 channels, the
# fastest of 4/8/16 x 2/4 at 4096 leaves (tools/fc_tail_bench.py, profiles/r03_fc_tail_bench.json)
FC2_KPARTS = 4
FC34_KPARTS = 2
# the FC tail below FC1_SPLIT_MIN_BATCH leaves (C2's 256; leaves % 256 == 0), also all on libazg's
# split GEMM: fc1 TRANSPOSED (W1 x A^T: the weights as the GEMM's rows, the leaves one column
# tile, so every weight tile is read once instead of once per 64-leaf row tile) in FC1T_KPARTS
# K-parts, azg_fc_act_t summing its transposed partials; fc2 and [fc3 | fc4] as before in
# FCS_KPARTS2 / FCS_KPARTS3 parts (short launches: more parts, fewer K stages each)
FC1T_KPARTS = 18
FCS_KPARTS2 = 16
FCS_KPARTS3 = 8
# ... the default (InferenceNet.fc_tail_small): with its epilogues loading every split-K part in flight
# (policy_value 14.8 -> 6.9 us, fc_act 6.1 -> 4.8 us per 256-leaf forward) it measured 1.037M exp/s at C2
# against 1.005M for the f32 hipBLASLt tail eager and 1.078M / 1.082M in graph replay, the same box
# (profiles/r05_bench_C2_tail_ab_*.json); before that, 1.02-1.06M over seven K-part choices against
# 1.10M.  No library GEMM is left in the C2 forward.
FC_SMALL_TAIL = True


class InflexionNNet(nn.Module):
    def __init__(self, n=7, depth=4, action_size=343, num_channels=512, dropout=0.3):
        super().__init__()
        c = num_channels
        self.n, self.depth, self.action_size = n, depth, action_size
        self.num_channels, self.dropout = c, dropout
        # creation order matters for manual_seed parity: conv1..4, bn1..4, fc1, fc_bn1, fc2, fc_bn2, fc3, fc4
        for i, (cin, pad) in enumerate([(depth, 1), (c, 1), (c, 0), (c, 0)], start=1):
            setattr(self, f"conv{i}", nn.Conv2d(cin, c, 3, stride=1, padding=pad))
        for i in range(1, 5):
            setattr(self, f"bn{i}", nn.BatchNorm2d(c))
        self.fc1 = nn.Linear(c * (n - 4) * (n - 4), 1024)
        self.fc_bn1 = nn.BatchNorm1d(1024)
        self.fc2 = nn.Linear(1024, 512)
        self.fc_bn2 = nn.BatchNorm1d(512)
        self.fc3 = nn.Linear(512, action_size)
        self.fc4 = nn.Linear(512, 1)

    def forward(self, s):
        x = s.view(-1, self.depth, self.n, self.n)
        for i in range(1, 5):
            x = F.relu(getattr(self, f"bn{i}")(getattr(self, f"conv{i}")(x)))
        x = x.reshape(x.shape[0], -1)
        x = F.dropout(F.relu(self.fc_bn1(self.fc1(x))), p=self.dropout, training=self.training)
        x = F.dropout(F.relu(self.fc_bn2(self.fc2(x))), p=self.dropout, training=self.training)
        return F.log_softmax(self.fc3(x), dim=1), torch.tanh(self.fc4(x))


def _addmm_relu(b, x, w):
    """relu(b + x w): one hipBLASLt GEMM with the bias and ReLU in its epilogue where
    torch has the fused op (torch._addmm_activation), else addmm + relu."""
    fused = getattr(torch, "_addmm_activation", None)
    if fused is not None:
        return fused(b, x, w)
    return torch.relu_(torch.addmm(b, x, w))


def _bias_relu_(x, b):
    """x = relu(x + b) in place on a channels_last CUDA tensor (libazg, one pass)."""
    import ctypes
    from . import _lib
    if not x.is_contiguous(memory_format=torch.channels_last):
        x = x.contiguous(memory_format=torch.channels_last)
    rows = x.numel() // x.shape[1]
    rc = _lib.lib().azg_bias_relu_nhwc(ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(b.data_ptr()), rows,
                                       x.shape[1], ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream))
    _lib.check(rc)
    return x


def _azg_conv3x3(x, wt, b, pad):
    """relu(conv3x3(x) + b) on a channels_last CUDA tensor by libazg's f32-MFMA
    implicit GEMM (azg_nn.hip); returns a channels_last tensor."""
    import ctypes
    from . import _lib
    if not x.is_contiguous(memory_format=torch.channels_last):
        x = x.contiguous(memory_format=torch.channels_last)
    B, C, H, _ = x.shape
    N = wt.shape[1]
    Ho = H + 2 * pad - 2
    y = torch.empty((B, N, Ho, Ho), device=x.device, dtype=torch.float32, memory_format=torch.channels_last)
    s = ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream)
    _lib.check(_lib.lib().azg_conv3x3_bias_relu_nhwc(ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(wt.data_ptr()),
                                                     ctypes.c_void_p(b.data_ptr()), ctypes.c_void_p(y.data_ptr()),
                                                     B, H, pad, C, N, s))
    return y


# Winograd F(m, 3) weight transforms G [m+2][3] (azg_winograd.hip holds B^T, A^T;
# azg_winograd_tables copies them out).  F(2,3): points 0, 1, -1; F(3,3): 0, 1, -1, 2;
# F(4,3): 0, 1, -1, 2, -1/2; F(5,3): 0, 1, -1, -1/2, -2, 3/2 -- B^T's rows scaled to
# small integers, their inverse scales in G (applied to the weights in f64).  The point
# sets keep the layer error at 1.2x (F(4,3)) and 2.6x (F(5,3)) F(3,3)'s
# (tools/wino_error_sim.py); the network's P, v stay within 1e-5 of the reference.
WINOGRAD_G = {2: [[1.0, 0.0, 0.0], [0.5, 0.5, 0.5], [0.5, -0.5, 0.5], [0.0, 0.0, 1.0]],
              3: [[0.5, 0.0, 0.0], [-0.5, -0.5, -0.5], [-1 / 6, 1 / 6, -1 / 6], [1 / 6, 1 / 3, 2 / 3],
                  [0.0, 0.0, 1.0]],
              4: [[0.5, 0.0, 0.0], [-1 / 6, -1 / 6, -1 / 6], [1 / 6, -1 / 6, 1 / 6], [1 / 30, 1 / 15, 2 / 15],
                  [-16 / 15, 8 / 15, -4 / 15], [0.0, 0.0, 0.5]],
              5: [[1 / 6, 0.0, 0.0], [-1 / 18, -1 / 18, -1 / 18], [1 / 10, -1 / 10, 1 / 10],
                  [-4 / 9, 2 / 9, -1 / 9], [-1 / 126, 1 / 63, -2 / 63], [4 / 105, 2 / 35, 3 / 35],
                  [0.0, 0.0, 0.25]]}


def winograd_seq(h_out):
    """Tile sides along an h_out-long output axis (azg_winograd.hip WSeq, mirrored by
    azg_winograd_layout): the fewest tiles of side <= 5, p = ceil(h/5), sides as equal
    as possible, the bigger first -- 7: [4, 3], 5: [5], 3: [3], 8: [4, 4], 6: [3, 3],
    4: [4], 9: [5, 4]; h = 1: one 2-tile, cropped."""
    if h_out < 2:
        return [2]
    p = (h_out + 4) // 5
    big = -(-h_out // p)
    nbig = h_out - p * (big - 1)
    return [big] * nbig + [big - 1] * (p - nbig)


def winograd_types(h_out):
    """(big, small) tile sides of an axis (kernel group order (big,big) (big,small)
    (small,big) (small,small))."""
    big = winograd_seq(h_out)[0]
    return big, big - 1


def winograd_groups(h_out):
    """Tile types of an h_out x h_out output in the kernels' order (big,big) (big,small)
    (small,big) (small,small), present ones only: [(ma, mb, points (ma+2)(mb+2), tiles
    per image)]."""
    seq = winograd_seq(h_out)
    big, small = winograd_types(h_out)
    out = []
    for ma, mb in ((big, big), (big, small), (small, big), (small, small)):
        n = seq.count(ma) * seq.count(mb)
        if n:
            out.append((ma, mb, (ma + 2) * (mb + 2), n))
    return out


def winograd_points(h_out):
    """Transformed points per image (GEMM rows per image): (sum of (m + 2))^2."""
    return sum(m + 2 for m in winograd_seq(h_out)) ** 2


def _winograd_u(w, h_out):
    """Winograd weights of a layer with an h_out x h_out output, the groups of
    winograd_groups one after another: U[e = (ma+2) a + b][c][k] = (G_ma g_kc G_mb^T)[a][b],
    formed in f64 and rounded once (G has entries like 1/6, 1/15).  [points][C][K]."""
    us = []
    for ma, mb, P, _ in winograd_groups(h_out):
        Ga = torch.tensor(WINOGRAD_G[ma], dtype=torch.float64, device=w.device)
        Gb = torch.tensor(WINOGRAD_G[mb], dtype=torch.float64, device=w.device)
        u = torch.einsum("ar,kcrs,bs->abck", Ga, w.detach().double(), Gb)
        us.append(u.reshape(P, w.shape[1], w.shape[0]))
    return torch.cat(us).float().contiguous()


def _split_u(u):
    """Split-GEMM weights: U scaled by 2^k (max |U| 2^k in (512, 1024], so U's low
    halves stay out of fp16 subnormals), split exactly as hi = fp16(U 2^k),
    lo = fp16(U 2^k - hi).  Returns (hi, lo) [points][C][K] fp16 and 2^-k."""
    amax = float(u.detach().abs().max())
    k = int(np.floor(np.log2(1024.0 / amax))) if amax > 0 else 0
    us = u.detach().double() * (2.0 ** k)
    hi = us.half()
    lo = (us - hi.double()).half()
    return hi, lo, 2.0 ** -k


def split2_rows(hi, lo):
    """[..., C] hi and lo halves -> [..., 2C] rows of 32-channel blocks [hi(32) | lo(32)]
    (azg.h AZG_WINO_SPLIT2, the split GEMM's operand layout)."""
    sh = hi.shape
    return torch.cat([hi.reshape(*sh[:-1], sh[-1] // 32, 32), lo.reshape(*sh[:-1], sh[-1] // 32, 32)],
                     dim=-1).reshape(*sh[:-1], 2 * sh[-1]).contiguous()


def split2_halves(rows):
    """Inverse of split2_rows: [..., 2C] -> (hi, lo) [..., C]."""
    sh = rows.shape
    b = rows.reshape(*sh[:-1], sh[-1] // 64, 64)
    return b[..., :32].reshape(*sh[:-1], sh[-1] // 2), b[..., 32:].reshape(*sh[:-1], sh[-1] // 2)


def _split_operands(u, gemm):
    """Operand B of the split GEMM form: "split" (libazg azg_split_gemm): U^T rows of
    32-channel blocks [hi(32) | lo(32)], [points][K][2C] (as V in AZG_WINO_SPLIT2);
    "split_blas" (hipBLASLt): [hi; hi; lo] stacked along C, [points][3C][K], to meet V's
    [hi | lo | hi] rows.  Returns (B, 2^-k)."""
    hi, lo, scale = _split_u(u)
    if gemm == "split":
        return split2_rows(hi.transpose(1, 2), lo.transpose(1, 2)), scale
    return torch.cat([hi, hi, lo], dim=1).contiguous(), scale


def _fold_bn(weight, bias, bn):
    """Eval-mode BatchNorm folded into the preceding conv/linear (f64 math)."""
    scale = bn.weight.double() / torch.sqrt(bn.running_var.double() + bn.eps)
    w = weight.double() * scale.reshape(-1, *([1] * (weight.dim() - 1)))
    b = (bias.double() - bn.running_mean.double()) * scale + bn.bias.double()
    return w.float(), b.float()


# Activation range the split-fp16 operands keep full precision in: an activation v is split
# into hi = fp16(v), lo = fp16(v - hi); for |v| < 2^-3 lo falls into fp16's subnormals and v
# keeps an absolute error of 2^-25 instead of a relative one of 2^-22, and |v| > 65504
# overflows (the range flag, check_range).  Layers whose BatchNorm puts the activations
# outside ACT_BAND are rescaled by a power of two so their estimate lands at ACT_TARGET.
ACT_BAND = (0.5, 1024.0)
ACT_TARGET = 8.0


def act_exponent(bn):
    """Power-of-two exponent e for the activations relu(BN(x)) of one layer: 0 if the
    BatchNorm's own estimate of their size, max over channels of beta + 3 |gamma| (on data
    like the running statistics' the pre-activation is N(beta, gamma^2) per channel), lies in
    ACT_BAND, else round(log2(ACT_TARGET / estimate)).  Random-init BatchNorm (gamma 1, beta 0)
    gives 3: unscaled.  A layer whose every channel is dead (estimate 0) stays unscaled."""
    est = float((bn.bias.detach().double() + 3.0 * bn.weight.detach().double().abs()).clamp_min(0.0).max())
    if est <= 0.0 or ACT_BAND[0] <= est <= ACT_BAND[1]:
        return 0
    return int(max(-30, min(30, round(np.log2(ACT_TARGET / est)))))


class InferenceNet(nn.Module):
    """Inference form of InflexionNNet for the leaf batches (eval semantics only).

    Every BatchNorm is folded into its conv/linear, activations stay NHWC
    (channels_last) end to end so the implicit-GEMM convolutions need no layout
    transposes, fc1's input columns are permuted from NCHW to NHWC flatten
    order, and the heads return what the engine consumes: P = softmax(fc3)
    (= exp(log_softmax), NNet.py:94) and v = tanh(fc4).  Same f32 arithmetic
    class as the reference; results agree with InflexionNNet to ~1e-6 relative
    (tests/test_nnet_cpu.py)."""

    outputs_probs = True

    def __init__(self, net: InflexionNNet, conv="winograd", gemm="split", small=None):
        """conv (conv2-4): "winograd" (default; Winograd F(5,3)/F(4,3)/F(3,3) tiles: libazg
        fused input / output transforms around one GEMM per transformed point, bias + ReLU
        in the output transform, 3.8x fewer multiply-adds), "miopen" (MIOpen implicit GEMM + one fused
        bias/ReLU pass), "azg" (libazg's f32-MFMA implicit GEMM with the bias/ReLU
        in its epilogue) or "auto" (per layer and input shape, whichever measured
        faster on first use).  All within the 1e-5 tolerance of the reference
        network (tests/test_gpu_nn.py); measured side by side in DESIGN.md 4.1.

        gemm (the Winograd GEMMs): "split" (default; each f32 operand split into
        fp16 hi + lo, hi*hi + lo*hi + hi*lo on the fp16 MFMA with f32 accumulation in
        libazg's hand-written GEMM: f32-accurate products -- measured error at or below
        the f32 GEMM's), "split_blas" (the same products as one hipBLASLt fp16 GEMM
        over [hi | lo | hi] rows) or "f32" (f32 MFMA GEMMs, hipBLASLt).

        small: up to SMALL_MAX_B leaves, run the whole forward on libazg's small-batch
        kernels (azg_small.hip) instead of MIOpen / hipBLASLt (None: SMALL_PATH) -- whatever
        `conv` says (small=False keeps a form's library path at a few leaves too)."""
        super().__init__()
        if conv not in ("miopen", "azg", "auto", "winograd"):
            raise ValueError(f"unknown conv implementation {conv!r}")
        if gemm not in ("split", "split_blas", "f32"):
            raise ValueError(f"unknown gemm form {gemm!r}")
        self.conv_impl = conv
        if gemm == "split" and (net.num_channels % 256 or net.num_channels % 32):
            gemm = "split_blas"  # libazg's split GEMM tiles K by 256
        self.gemm = gemm
        self.mscale = {}  # Winograd layer -> 2^-k undoing the split operand's scale
        self._choices = {}
        self._ws = None  # Winograd V / M workspace, grown to the largest layer seen
        # up to SMALL_MAX_B leaves: the whole forward on libazg's small-batch kernels
        # (azg_small.hip) instead of MIOpen / hipBLASLt
        self.small_path = SMALL_PATH if small is None else bool(small)
        self._init_args = (conv, gemm, small)
        self.h_out = {}  # output side per conv layer
        self.fuse_transforms = True  # conv2->3->4: output + next input transform in one pass
        self.n, self.depth, c = net.n, net.depth, net.num_channels
        self.pads = []
        # power-of-two activation scales (act_exponent): layer i's folded weights and bias carry
        # 2^(e_i - e_(i-1)) and 2^e_i, so its output is 2^e_i relu(BN(conv)) exactly (ReLU is
        # positively homogeneous and the scalings are exact in f32); [fc3 | fc4] undo the last one
        self.act_exp = {}
        e_prev = 0
        h = net.n  # input side of conv i
        for i in range(1, 5):
            conv_i, bn = getattr(net, f"conv{i}"), getattr(net, f"bn{i}")
            h_out = h + 2 * conv_i.padding[0] - 2
            w, b = _fold_bn(conv_i.weight.detach(), conv_i.bias.detach(), bn)
            e = act_exponent(bn)
            w, b = w * 2.0 ** (e - e_prev), b * 2.0 ** e
            self.act_exp[i], e_prev = e, e
            self.register_buffer(f"w{i}", w.contiguous(memory_format=torch.channels_last))
            self.register_buffer(f"b{i}", b)
            # [9*Cin, Cout] k-major copy for the libazg implicit GEMM (k = (dy*3+dx)*Cin + c)
            self.register_buffer(f"wt{i}", w.permute(2, 3, 1, 0).reshape(-1, w.shape[0]).contiguous())
            if i == 1:
                self.register_buffer("w1c", w.contiguous())  # [K][depth][3][3] for the fused front end
            self.h_out[i] = h_out
            if i > 1 and conv in ("winograd", "auto"):
                u = _winograd_u(w, h_out)
                self.register_buffer(f"u{i}", u)
                if gemm != "f32":
                    ub, self.mscale[i] = _split_operands(u, gemm)
                    self.register_buffer(f"us_{i}", ub)
            self.pads.append(conv_i.padding[0])
            h = h_out
        s = net.n - 4
        w1, b1 = _fold_bn(net.fc1.weight.detach(), net.fc1.bias.detach(), net.fc_bn1)
        e = act_exponent(net.fc_bn1)
        w1, b1 = w1 * 2.0 ** (e - e_prev), b1 * 2.0 ** e
        self.act_exp["fc1"], e_prev = e, e
        w1 = w1.reshape(-1, c, s, s).permute(0, 2, 3, 1).reshape(w1.shape[0], -1)  # (c,h,w) -> (h,w,c)
        self.register_buffer("fw1", w1.contiguous())
        # fc1 as a split-fp16 GEMM (with a split GEMM form): conv4's output transform
        # writes the flattened activation as [hi | lo | hi] rows, fc1's weights are
        # stacked [hi; hi; lo] (scaled by a power of two, undone with the bias)
        self.fc1_split = gemm != "f32"
        # fc1 on libazg's split GEMM as a split-K GEMM of FC1_KPARTS parts (the parts are
        # the GEMM's "points": ~256 output tiles at 4096 leaves instead of 64), its A
        # operand written by conv4's output transform in [parts][leaves][chunk] blocks
        width = w1.shape[1]
        self.fc1_kparts = FC1_KPARTS if (gemm == "split" and width % (64 * FC1_KPARTS) == 0
                                         and w1.shape[0] % 256 == 0) else 0
        if self.fc1_split:
            whi, wlo, self.fc1_scale = _split_u(w1.t().unsqueeze(0))
            self.register_buffer("fw1_s", torch.cat([whi, whi, wlo], dim=1).contiguous())
            if self.fc1_kparts:
                kp, n1 = self.fc1_kparts, w1.shape[0]
                hp = whi[0].t().reshape(n1, kp, width // kp).transpose(0, 1)
                lp = wlo[0].t().reshape(n1, kp, width // kp).transpose(0, 1)
                self.register_buffer("fw1_sk", split2_rows(hp, lp))  # [parts][N][2 chunk]
        self.register_buffer("fb1", b1)
        w2, b2 = _fold_bn(net.fc2.weight.detach(), net.fc2.bias.detach(), net.fc_bn2)
        e = act_exponent(net.fc_bn2)
        w2, b2 = w2 * 2.0 ** (e - e_prev), b2 * 2.0 ** e
        self.act_exp["fc2"], e_prev = e, e
        self.register_buffer("fw2", w2.contiguous())
        self.register_buffer("fb2", b2)
        self.register_buffer("fw3", net.fc3.weight.detach() * 2.0 ** -e_prev)
        self.register_buffer("fb3", net.fc3.bias.detach().clone())
        self.register_buffer("fw4", net.fc4.weight.detach() * 2.0 ** -e_prev)
        self.register_buffer("fb4", net.fc4.bias.detach().clone())
        # fc3 and fc4 read the same activation: one GEMM over their stacked rows
        self.register_buffer("fw34", torch.cat([self.fw3, self.fw4], dim=0).contiguous())
        self.register_buffer("fb34", torch.cat([self.fb3, self.fb4]).contiguous())
        # with the split form, fc2 and [fc3 | fc4] are split GEMMs too: each layer's bias +
        # ReLU epilogue writes the next layer's [hi | lo | hi] rows (azg_fc_act_split), and
        # one kernel turns the stacked fc3 | fc4 output into P and v (azg_policy_value)
        if self.fc1_split:
            whi, wlo, self.fc2_scale = _split_u(w2.t().unsqueeze(0))
            self.register_buffer("fw2_s", torch.cat([whi, whi, wlo], dim=1).contiguous())
            whi, wlo, self.fc34_scale = _split_u(self.fw34.t().unsqueeze(0))
            self.register_buffer("fw34_s", torch.cat([whi, whi, wlo], dim=1).contiguous())
        # the whole FC tail on libazg's split GEMM (fc1 split-K as above, then fc2 and the
        # stacked [fc3 | fc4] as split-K GEMMs whose A operands the epilogues write in the
        # split GEMM's own layout, azg_fc_act AZG_WINO_SPLIT2): no library GEMM in the forward
        n2, n34 = w2.shape[0], self.fw34.shape[0]
        self.fc_tail_azg = bool(self.fc1_kparts) and n2 % 256 == 0 and (w2.shape[1] // FC2_KPARTS) % 64 == 0 \
            and (n2 // FC34_KPARTS) % 64 == 0 and w2.shape[1] % FC2_KPARTS == 0 and n2 % FC34_KPARTS == 0
        if self.fc_tail_azg:
            self.fc2_kparts, self.fc34_kparts = FC2_KPARTS, FC34_KPARTS
            self.register_buffer("fw2_sk", self._split_k_weights(w2, FC2_KPARTS, self.fc2_scale))
            n34p = -(-n34 // 256) * 256  # the split GEMM's 256-column tiles: zero weights past fc4
            w34 = torch.zeros((n34p, self.fw34.shape[1]), dtype=self.fw34.dtype, device=self.fw34.device)
            w34[:n34] = self.fw34
            self.register_buffer("fw34_sk", self._split_k_weights(w34, FC34_KPARTS, self.fc34_scale))
            # the small-batch tail (FC1T_KPARTS, FCS_KPARTS2 / 3; _fc_split_small)
            w1w = w1.shape[1]
            small_ok = (w1w % (64 * FC1T_KPARTS) == 0 and w1.shape[0] % 64 == 0
                        and w2.shape[1] % (64 * FCS_KPARTS2) == 0 and n2 % (64 * FCS_KPARTS3) == 0)
            self.fc_tail_small = small_ok and FC_SMALL_TAIL
            if small_ok:
                self.register_buffer("fw1_skT", self._split_k_weights(w1, FC1T_KPARTS, self.fc1_scale))
                self.register_buffer("fw2_skS", self._split_k_weights(w2, FCS_KPARTS2, self.fc2_scale))
                self.register_buffer("fw34_skS", self._split_k_weights(w34, FCS_KPARTS3, self.fc34_scale))
        else:
            self.fc_tail_small = False
        # sticky device flag: a split-GEMM operand fp16 could not hold (checked by check_range).
        # It lives where the kernels run: the transforms set it with a device atomic, so a
        # host-memory flag would fault the GPU the first time an operand overflowed.
        self.register_buffer("overflow", torch.zeros(1, dtype=torch.int32, device=self.w1.device))

    @staticmethod
    def _split_k_weights(w, kp, scale):
        """[N][C] f32 weights -> the B operand of a kp-part split-K split GEMM: [kp][N][2 C / kp]
        32-channel [hi | lo] blocks of W 2^k (the scale 2^-k _split_u picked for the same W)."""
        us = w.detach().double().t() / scale  # [C][N], times 2^k
        hi = us.half()
        lo = (us - hi.double()).half()
        n, c = w.shape
        hp = hi.t().reshape(n, kp, c // kp).transpose(0, 1)
        lp = lo.t().reshape(n, kp, c // kp).transpose(0, 1)
        return split2_rows(hp, lp)

    def set_winograd_layer(self, i, w, h_out):
        """Replace conv i's Winograd weights by w [K][C][3][3] (BN already folded) for an
        h_out x h_out output."""
        self.h_out[i] = h_out
        u = _winograd_u(w, h_out).to(self.w1.device)
        setattr(self, f"u{i}", u)
        if self.gemm != "f32":
            ub, self.mscale[i] = _split_operands(u, self.gemm)
            setattr(self, f"us_{i}", ub)

    def check_range(self):
        """Raise if any split-GEMM operand since the last call was out of fp16 range
        (|v| > 65504 or NaN): the GEMM would have been wrong, not just inexact."""
        if self.gemm != "f32" and int(self.overflow.item()) != 0:
            self.overflow.zero_()
            raise FloatingPointError("Winograd split-GEMM operand out of fp16 range; use InferenceNet(gemm='f32')")

    # optional hooks used by bench.py to bracket work with HIP events on the current
    # stream: conv_hook(layer_index, "start"|"stop") around each convolution,
    # kernel_hook(kind, layer_index, "start"|"stop", flops) around each libazg launch of
    # kind "gemm" (azg_split_gemm: conv2-4 and fc1, with the launch's executed fp16 MFMA
    # FLOPs, 3 products per f32 multiply-add) or "transform" (the Winograd transforms)
    conv_hook = None
    kernel_hook = None

    def _khook(self, kind, i, what, flops=0.0, variant=None):
        """flops (on "stop"): the executed MFMA FLOPs of a GEMM launch; variant: the split
        GEMM schedule azg_split_gemm picked for it (4 persistent 256-row tiles, 17 / 18
        128 / 64-row tiles)."""
        if self.kernel_hook is not None:
            self.kernel_hook(kind, i, what, flops, variant)

    @staticmethod
    def _gemm_pick(runs_pts, runs_rows, k):
        import ctypes
        from . import _lib
        n = len(runs_pts)
        return _lib.lib().azg_split_gemm_pick(n, (ctypes.c_int32 * n)(*runs_pts), (ctypes.c_int32 * n)(*runs_rows), k)

    def _conv_miopen(self, x, i, pad):
        # MIOpen conv without bias, then one HIP pass: bias + ReLU in place (azg_nn.hip)
        x = F.conv2d(x, getattr(self, f"w{i}"), None, padding=pad)
        return _bias_relu_(x, getattr(self, f"b{i}"))

    def _conv_azg(self, x, i, pad):
        # bias + ReLU inside the libazg conv's epilogue
        return _azg_conv3x3(x, getattr(self, f"wt{i}"), getattr(self, f"b{i}"), pad)

    def _v_words(self, rows, C):
        """f32 words of a V with `rows` rows: f32 rows of C, fp16 rows of 2C (split) or 3C (split_blas)."""
        return rows * C if self.gemm in ("f32", "split") else (3 * rows * C + 1) // 2

    def _gemm_runs(self, i):
        """[points, tiles per image] runs of layer i's GEMMs (tile groups with equal tiles
        per image merged): 7x7 output: 1 run, 5x5: 1, 3x3: 1."""
        runs = []
        for _, _, P, n in winograd_groups(self.h_out[i]):
            if runs and runs[-1][1] == n:
                runs[-1][0] += P
            else:
                runs.append([P, n])
        return runs

    def _wino_need(self, i, B, C, fuse_next):
        """Workspace words layer i needs: (its V, or the next layer's V when larger and fused; its M)."""
        K = getattr(self, f"u{i}").shape[2]
        rows = B * winograd_points(self.h_out[i])
        need_v = self._v_words(rows, C)
        if fuse_next:
            need_v = max(need_v, self._v_words(B * winograd_points(self.h_out[i + 1]), K))
        return need_v, rows * K

    def _ensure_ws(self, need, dev):
        if self._ws is None or self._ws[0].numel() < need[0] or self._ws[1].numel() < need[1]:
            self._ws = (torch.empty(need[0], device=dev), torch.empty(need[1], device=dev))

    def _ws_fits(self, need):
        return self._ws is not None and self._ws[0].numel() >= need[0] and self._ws[1].numel() >= need[1]

    def _vfmt(self):
        """(azg.h AZG_WINO_* format of V, overflow flag pointer)."""
        if self.gemm == "f32":
            return 0, None
        return (2 if self.gemm == "split" else 1), self._overflow_ptr()

    def _overflow_ptr(self):
        """Device address of the range flag, on the device of the weights the kernels read."""
        if self.overflow.device != self.w1.device:
            self.overflow = self.overflow.to(self.w1.device)
        if not self.overflow.is_cuda:
            raise RuntimeError("InferenceNet's kernels need its weights on the GPU")
        return self.overflow.data_ptr()

    def _first_winograd(self, s):
        """conv1 + bias + ReLU + conv2's Winograd input transform straight from the NCHW
        planes (azg_winograd_first_nchw); conv2's V is left in the workspace."""
        import ctypes
        from . import _lib
        B = s.shape[0]
        C = self.w1c.shape[0]
        self._ensure_ws(self._wino_need(2, B, C, True), s.device)
        st = ctypes.c_void_p(torch.cuda.current_stream(s.device).cuda_stream)
        fmt, ovf = self._vfmt()
        self._khook("transform", 1, "start")
        _lib.check(_lib.lib().azg_winograd_first_nchw(
            ctypes.c_void_p(s.data_ptr()), ctypes.c_void_p(self.w1c.data_ptr()), ctypes.c_void_p(self.b1.data_ptr()),
            ctypes.c_void_p(self._ws[0].data_ptr()), B, self.depth, self.n, C, fmt, ctypes.c_void_p(ovf), st))
        self._khook("transform", 1, "stop")

    def _winograd_gemms(self, i, B, C, K):
        """M = V x U for every transformed point of layer i, by runs of tile groups with
        equal tiles per image (7x7: 1 run, 5x5: 1, 3x3: 1): one libazg azg_split_gemm
        launch for all runs ("split"), or one torch.bmm (hipBLASLt) per run."""
        runs = self._gemm_runs(i)
        if self.gemm == "split":
            import ctypes
            from . import _lib
            pts = (ctypes.c_int32 * len(runs))(*[P for P, _ in runs])
            rows = (ctypes.c_int32 * len(runs))(*[B * n for _, n in runs])
            self._khook("gemm", i, "start")
            _lib.check(_lib.lib().azg_split_gemm(
                ctypes.c_void_p(self._ws[0].data_ptr()), ctypes.c_void_p(getattr(self, f"us_{i}").data_ptr()),
                ctypes.c_void_p(self._ws[1].data_ptr()), len(runs), pts, rows, C, K,
                ctypes.c_void_p(torch.cuda.current_stream(self._ws[0].device).cuda_stream)))
            self._khook("gemm", i, "stop", 3.0 * 2 * C * K * sum(P * B * n for P, n in runs),
                        self._gemm_pick([P for P, _ in runs], [B * n for _, n in runs], K) if self.kernel_hook else None)
            return
        split = self.gemm == "split_blas"
        W = 3 * C if split else C
        Vflat = self._ws[0].view(torch.float16) if split else self._ws[0]
        U = getattr(self, f"us_{i}") if split else getattr(self, f"u{i}")
        row = pt = 0
        for P, n in runs:
            T = B * n
            V = Vflat[row * W:(row + P * T) * W].view(P, T, W)
            M = self._ws[1][row * K:(row + P * T) * K].view(P, T, K)
            if split:
                torch.bmm(V, U[pt:pt + P], out_dtype=torch.float32, out=M)
            else:
                torch.bmm(V, U[pt:pt + P], out=M)
            row += P * T
            pt += P

    def _conv_winograd(self, x, i, pad, in_bias=None, carried=False, B=None, H=None, fuse_next=False,
                       split_out=False):
        """Winograd layer i (F(5,3)/F(4,3)/F(3,3) tiles, azg_winograd.hip): libazg input
        transform (or, with carried=True, the V the previous layer's fused transform left
        in the workspace), the GEMMs (_winograd_gemms), then either the output transform
        with bias + ReLU (returns the NHWC activation) or, with fuse_next, the fused
        output / next-input transform writing layer i+1's V (returns None)."""
        import ctypes
        from . import _lib
        if not carried:
            if not x.is_contiguous(memory_format=torch.channels_last):
                x = x.contiguous(memory_format=torch.channels_last)
            B, C, H, _ = x.shape
            dev = x.device
        else:
            C = getattr(self, f"u{i}").shape[1]
            dev = self._ws[0].device
        K = getattr(self, f"u{i}").shape[2]
        Ho = H + 2 * pad - 2
        if Ho != self.h_out[i]:
            raise ValueError(f"conv{i}: input side {H} gives {Ho}x{Ho} outputs, the weights are for {self.h_out[i]}")
        need = self._wino_need(i, B, C, fuse_next)
        if not carried:
            self._ensure_ws(need, dev)
        elif not self._ws_fits(need):
            raise RuntimeError("Winograd workspace too small for a carried layer")
        mscale = self.mscale[i] if self.gemm != "f32" else 1.0
        s = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        L = _lib.lib()
        bias = ctypes.c_void_p(getattr(self, f"b{i}").data_ptr())
        fmt, ovf = self._vfmt()
        V, M = ctypes.c_void_p(self._ws[0].data_ptr()), ctypes.c_void_p(self._ws[1].data_ptr())
        if not carried:
            ib = ctypes.c_void_p(in_bias.data_ptr()) if in_bias is not None else None
            _lib.check(L.azg_winograd_in_nhwc(ctypes.c_void_p(x.data_ptr()), ib, V, B, H, pad, C, fmt,
                                              ctypes.c_void_p(ovf), s))
        self._winograd_gemms(i, B, C, K)
        if fuse_next:
            self._khook("transform", i, "start")
            _lib.check(L.azg_winograd_mid_nhwc(M, bias, V, B, Ho, K, mscale, fmt, ctypes.c_void_p(ovf), s))
            self._khook("transform", i, "stop")
            return None
        if split_out:
            # the flattened NHWC activation as fc1's A operand: [parts][B][chunk] split2 blocks
            # for libazg's split-K GEMM, else one [hi | lo | hi] fp16 row per image (hipBLASLt)
            # (the small tail's part count from its own buffer: the one it was split with)
            kp = self.fc1_kparts if B >= FC1_SPLIT_MIN_BATCH else self.fw1_skT.shape[0]
            y = torch.empty((B, (2 if kp else 3) * Ho * Ho * K), device=dev, dtype=torch.float16)
            self._khook("transform", i, "start")
            _lib.check(L.azg_winograd_out_split(M, bias, ctypes.c_void_p(y.data_ptr()), B, Ho, K, 1, mscale,
                                                2 if kp else 1, max(kp, 1),
                                                ctypes.c_void_p(self._overflow_ptr()), s))
            self._khook("transform", i, "stop")
            return y
        y = torch.empty((B, K, Ho, Ho), device=dev, dtype=torch.float32, memory_format=torch.channels_last)
        _lib.check(L.azg_winograd_out_nhwc(M, bias, ctypes.c_void_p(y.data_ptr()), B, Ho, K, 1, mscale, s))
        return y

    def _pick(self, x, i, pad):
        """conv="auto": time both implementations once per (layer, input shape) and
        keep the faster (like cudnn.benchmark).  Never inside a graph capture: an
        unmeasured shape there takes MIOpen."""
        key = (i, tuple(x.shape))
        choice = self._choices.get(key)
        if choice is not None:
            return choice
        if torch.cuda.is_current_stream_capturing():
            return "miopen"
        best = None
        for name, fn in (("miopen", self._conv_miopen), ("azg", self._conv_azg), ("winograd", self._conv_winograd)):
            for _ in range(2):
                fn(x, i, pad)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            for _ in range(3):
                fn(x, i, pad)
            ev[1].record()
            ev[1].synchronize()
            ms = ev[0].elapsed_time(ev[1])
            if best is None or ms < best[1]:
                best = (name, ms)
        self._choices[key] = best[0]
        return best[0]

    def _fc_split(self, a):
        """The FC tail on split-fp16 GEMMs (azg_heads.hip): fc1 (+ folded fc_bn1) + ReLU,
        fc2 (+ fc_bn2) + ReLU, [fc3 | fc4] as hi.Wh + lo.Wh + hi.Wl on the fp16 MFMA
        (hipBLASLt, f32 accumulation), each epilogue writing the next GEMM's [hi | lo | hi]
        rows; then P = softmax(fc3), v = tanh(fc4).  fc1 runs on libazg's split GEMM as a
        split-K GEMM (fc1_kparts > 0) or on hipBLASLt.  a: conv4's flattened activation
        (azg_winograd_out_split) as [parts][B][chunk] split2 blocks or [B, 3 * 4608] fp16 rows."""
        import ctypes
        from . import _lib
        L = _lib.lib()
        B, dev = a.shape[0], a.device
        st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        ovf = ctypes.c_void_p(self._overflow_ptr())
        if self.fc_tail_small and B < FC1_SPLIT_MIN_BATCH:
            return self._fc_split_small(a, B, dev, st, ovf)
        if self.fc_tail_azg and self.fc1_kparts:
            return self._fc_split_azg(a, B, dev, st, ovf)
        for layer, (w, b, scale) in enumerate(((self.fw1_s, self.fb1, self.fc1_scale),
                                               (self.fw2_s, self.fb2, self.fc2_scale))):
            n = w.shape[2]
            kp = self.fc1_kparts if layer == 0 else 0
            if kp:  # fc1: libazg split GEMM, the K parts as points, partial products summed below
                m = torch.empty((kp, B, n), device=dev, dtype=torch.float32)
                chunk = a.shape[1] // (2 * kp)
                pts, rows = (ctypes.c_int32 * 1)(kp), (ctypes.c_int32 * 1)(B)
                self._khook("gemm", 5, "start")
                _lib.check(L.azg_split_gemm(ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(self.fw1_sk.data_ptr()),
                                            ctypes.c_void_p(m.data_ptr()), 1, pts, rows, chunk, n, st))
                self._khook("gemm", 5, "stop", 3.0 * 2 * kp * chunk * n * B,
                            self._gemm_pick([kp], [B], n) if self.kernel_hook else None)
            else:
                m = torch.empty((1, B, n), device=dev, dtype=torch.float32)
                torch.bmm(a.unsqueeze(0), w, out_dtype=torch.float32, out=m)
            a = torch.empty((B, 3 * n), device=dev, dtype=torch.float16)
            _lib.check(L.azg_fc_act_split(ctypes.c_void_p(m.data_ptr()), max(kp, 1), B * n,
                                          ctypes.c_void_p(b.data_ptr()), scale, ctypes.c_void_p(a.data_ptr()), B, n,
                                          1, ovf, st))
        n = self.fw34_s.shape[2]
        m = torch.empty((1, B, n), device=dev, dtype=torch.float32)
        torch.bmm(a.unsqueeze(0), self.fw34_s, out_dtype=torch.float32, out=m)
        A = n - 1
        p = torch.empty((B, A), device=dev, dtype=torch.float32)
        v = torch.empty((B, 1), device=dev, dtype=torch.float32)
        _lib.check(L.azg_policy_value(ctypes.c_void_p(m.data_ptr()), n, ctypes.c_void_p(self.fb34.data_ptr()),
                                      self.fc34_scale, ctypes.c_void_p(p.data_ptr()), ctypes.c_void_p(v.data_ptr()),
                                      B, A, st))
        return p, v

    def _fc_split_azg(self, a, B, dev, st, ovf):
        """The FC tail as three split-K libazg split GEMMs (fc1, fc2, [fc3 | fc4] padded to 512
        columns), each epilogue (azg_fc_act) summing the previous GEMM's parts in order,
        adding the folded bias, applying ReLU and writing the next GEMM's split2 K-parts;
        azg_policy_value_parts sums the last GEMM's parts into P = softmax, v = tanh."""
        import ctypes
        from . import _lib
        L = _lib.lib()

        def gemm(layer, A_, W, kp, n):
            c = A_.shape[-1] // (2 * kp) if A_.dim() == 2 else A_.shape[-1] // 2
            m = torch.empty((kp, B, n), device=dev, dtype=torch.float32)
            pts, rows = (ctypes.c_int32 * 1)(kp), (ctypes.c_int32 * 1)(B)
            self._khook("gemm", layer, "start")
            _lib.check(L.azg_split_gemm(ctypes.c_void_p(A_.data_ptr()), ctypes.c_void_p(W.data_ptr()),
                                        ctypes.c_void_p(m.data_ptr()), 1, pts, rows, c, n, st))
            self._khook("gemm", layer, "stop", 3.0 * 2 * kp * c * n * B,
                        self._gemm_pick([kp], [B], n) if self.kernel_hook else None)
            return m

        def act(m, kp_in, bias, scale, kp_out):
            n = m.shape[2]
            out = torch.empty((kp_out, B, 2 * n // kp_out), device=dev, dtype=torch.float16)
            _lib.check(L.azg_fc_act(ctypes.c_void_p(m.data_ptr()), kp_in, B * n, ctypes.c_void_p(bias.data_ptr()),
                                    scale, ctypes.c_void_p(out.data_ptr()), B, n, 1, 2, kp_out, ovf, st))
            return out

        kp1, kp2, kp3 = self.fc1_kparts, self.fc2_kparts, self.fc34_kparts
        m1 = gemm(5, a, self.fw1_sk, kp1, self.fw1_sk.shape[1])
        a2 = act(m1, kp1, self.fb1, self.fc1_scale, kp2)
        m2 = gemm(6, a2, self.fw2_sk, kp2, self.fw2_sk.shape[1])
        a3 = act(m2, kp2, self.fb2, self.fc2_scale, kp3)
        m3 = gemm(7, a3, self.fw34_sk, kp3, self.fw34_sk.shape[1])
        A = self.fw34.shape[0] - 1
        p = torch.empty((B, A), device=dev, dtype=torch.float32)
        v = torch.empty((B, 1), device=dev, dtype=torch.float32)
        n3 = m3.shape[2]
        _lib.check(L.azg_policy_value_parts(ctypes.c_void_p(m3.data_ptr()), kp3, B * n3, n3,
                                            ctypes.c_void_p(self.fb34.data_ptr()), self.fc34_scale,
                                            ctypes.c_void_p(p.data_ptr()), ctypes.c_void_p(v.data_ptr()), B, A, st))
        return p, v

    def _fc_split_small(self, a, B, dev, st, ovf):
        """The FC tail below FC1_SPLIT_MIN_BATCH leaves (leaves % 256 == 0, C2's 256): fc1 as the
        transposed split-K GEMM M1^T [parts][1024][B] = W1 A^T (the weights the rows, the leaves one
        256-column tile: each weight tile read once), azg_fc_act_t summing its parts in order into
        fc2's split2 K-parts; fc2 and [fc3 | fc4] as _fc_split_azg's, in FCS_KPARTS2 / 3 parts."""
        import ctypes
        from . import _lib
        L = _lib.lib()
        # the part counts the buffers were split with (not the module globals, which a bench or test may
        # have changed since this form was built)
        kp1, kp2, kp3 = self.fw1_skT.shape[0], self.fw2_skS.shape[0], self.fw34_skS.shape[0]
        n1, c1 = self.fw1_skT.shape[1], self.fw1_skT.shape[2] // 2
        m1 = torch.empty((kp1, n1, B), device=dev, dtype=torch.float32)
        pts, rows = (ctypes.c_int32 * 1)(kp1), (ctypes.c_int32 * 1)(n1)
        self._khook("gemm", 5, "start")
        _lib.check(L.azg_split_gemm(ctypes.c_void_p(self.fw1_skT.data_ptr()), ctypes.c_void_p(a.data_ptr()),
                                    ctypes.c_void_p(m1.data_ptr()), 1, pts, rows, c1, B, st))
        self._khook("gemm", 5, "stop", 3.0 * 2 * kp1 * c1 * n1 * B,
                    self._gemm_pick([kp1], [n1], B) if self.kernel_hook else None)
        n2 = self.fw2_skS.shape[1]
        a2 = torch.empty((kp2, B, 2 * n1 // kp2), device=dev, dtype=torch.float16)
        _lib.check(L.azg_fc_act_t(ctypes.c_void_p(m1.data_ptr()), kp1, n1 * B, ctypes.c_void_p(self.fb1.data_ptr()),
                                  self.fc1_scale, ctypes.c_void_p(a2.data_ptr()), B, n1, 1, kp2, ovf, st))

        def gemm(layer, A_, W, kp, n):
            c = A_.shape[-1] // 2
            m = torch.empty((kp, B, n), device=dev, dtype=torch.float32)
            pts, rows = (ctypes.c_int32 * 1)(kp), (ctypes.c_int32 * 1)(B)
            self._khook("gemm", layer, "start")
            _lib.check(L.azg_split_gemm(ctypes.c_void_p(A_.data_ptr()), ctypes.c_void_p(W.data_ptr()),
                                        ctypes.c_void_p(m.data_ptr()), 1, pts, rows, c, n, st))
            self._khook("gemm", layer, "stop", 3.0 * 2 * kp * c * n * B,
                        self._gemm_pick([kp], [B], n) if self.kernel_hook else None)
            return m
        m2 = gemm(6, a2, self.fw2_skS, kp2, n2)
        a3 = torch.empty((kp3, B, 2 * n2 // kp3), device=dev, dtype=torch.float16)
        _lib.check(L.azg_fc_act(ctypes.c_void_p(m2.data_ptr()), kp2, B * n2, ctypes.c_void_p(self.fb2.data_ptr()),
                                self.fc2_scale, ctypes.c_void_p(a3.data_ptr()), B, n2, 1, 2, kp3, ovf, st))
        m3 = gemm(7, a3, self.fw34_skS, kp3, self.fw34_skS.shape[1])
        A = self.fw34.shape[0] - 1
        p = torch.empty((B, A), device=dev, dtype=torch.float32)
        v = torch.empty((B, 1), device=dev, dtype=torch.float32)
        n3 = m3.shape[2]
        _lib.check(L.azg_policy_value_parts(ctypes.c_void_p(m3.data_ptr()), kp3, B * n3, n3,
                                            ctypes.c_void_p(self.fb34.data_ptr()), self.fc34_scale,
                                            ctypes.c_void_p(p.data_ptr()), ctypes.c_void_p(v.data_ptr()), B, A, st))
        return p, v

    def refresh_from(self, net):
        """Re-fold `net`'s current weights into this form's own buffers, in place (the same
        storage, so HIP graphs captured over this evaluator stay valid; the small-batch path
        passes no weight-dependent scalars to its kernels)."""
        fresh = InferenceNet(net, *self._init_args)
        for name, buf in fresh.named_buffers():
            if name == "overflow":
                continue
            getattr(self, name).copy_(buf)
        self.mscale = dict(fresh.mscale)
        for k in ("fc1_scale", "fc2_scale", "fc34_scale"):
            if hasattr(fresh, k):
                setattr(self, k, getattr(fresh, k))

    def _forward_small(self, planes):
        """The forward at up to SMALL_MAX_B leaves on libazg's small-batch kernels
        (azg_small.hip): conv1-4 (+ folded BN, bias, ReLU) from the NCHW leaf planes to NHWC
        rows, fc1 / fc2 (+ ReLU), [fc3 | fc4], then azg_policy_value's softmax / tanh."""
        import ctypes
        from . import _lib
        L = _lib.lib()
        planes = planes.contiguous()
        B, n, C = planes.shape[0], self.n, self.w1.shape[0]
        dev = planes.device
        st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        x, strides, H, cin = planes, (self.depth * n * n, n, 1, n * n), n, self.depth
        # the split-K convolutions' partial sums and per-channel-group tickets (zero between launches;
        # the last word is the heads kernel's)
        need = 8 * C * SMALL_MAX_B * n * n  # (azg_small.hip SK_KG = 8 K-parts)
        if getattr(self, "_small_work", None) is None or self._small_work.numel() < need \
                or self._small_work.device != dev:
            self._small_work = torch.empty(need, device=dev, dtype=torch.float32)
            self._small_tickets = torch.zeros(max(C // 8, 1) + 1, device=dev, dtype=torch.int32)
        work, tickets = self._small_work, self._small_tickets
        x, H = self._convs_small(planes, B, dev, st, work, tickets)
        feat = H * H * C  # NHWC flatten (fw1's column order)

        def fc(x, ldx, w, b, relu):
            N, K = w.shape
            out = torch.empty((B, N), device=dev, dtype=torch.float32)
            _lib.check(L.azg_small_fc(ctypes.c_void_p(x.data_ptr()), ldx, B, ctypes.c_void_p(w.data_ptr()), K, N,
                                      ctypes.c_void_p(b.data_ptr()) if b is not None else None, int(relu),
                                      ctypes.c_void_p(out.data_ptr()), N, st))
            return out
        h1 = fc(x, feat, self.fw1, self.fb1, True)
        h2 = fc(h1, h1.shape[1], self.fw2, self.fb2, True)
        A = self.fw3.shape[0]
        p = torch.empty((B, A), device=dev, dtype=torch.float32)
        v = torch.empty((B, 1), device=dev, dtype=torch.float32)
        logits = torch.empty((B, A + 1), device=dev, dtype=torch.float32)
        _lib.check(L.azg_small_heads(ctypes.c_void_p(h2.data_ptr()), h2.shape[1], B, ctypes.c_void_p(self.fw34.data_ptr()),
                                     self.fw34.shape[1], A, ctypes.c_void_p(self.fb34.data_ptr()),
                                     ctypes.c_void_p(logits.data_ptr()), ctypes.c_void_p(p.data_ptr()),
                                     ctypes.c_void_p(v.data_ptr()),
                                     ctypes.c_void_p(tickets.data_ptr() + 4 * (tickets.numel() - 1)), st))
        return p, v

    def _convs_small(self, planes, B, dev, st, work, tickets):
        """conv1-4 at up to SMALL_MAX_B leaves (azg_small_conv12 + azg_small_conv3x3): NHWC rows of
        conv4's output and its side."""
        import ctypes
        from . import _lib
        L = _lib.lib()
        n, C = self.n, self.w1.shape[0]
        wp, tp = ctypes.c_void_p(work.data_ptr()), ctypes.c_void_p(tickets.data_ptr())
        x, strides, H, cin, first = planes, (self.depth * n * n, n, 1, n * n), n, self.depth, 1
        if self.depth <= 4 and 6 <= n <= 8 and C % 16 == 0 and self.pads[:2] == [1, 1] \
                and n * n * (C // 4 + 4) * 4 + 72 * C + 16384 <= 96 * 1024:  # azg_small_conv12's LDS (4 K-parts)
            # conv1 + conv2 in one launch
            y = torch.empty((B * n * n, C), device=dev, dtype=torch.float32)
            _lib.check(L.azg_small_conv12(ctypes.c_void_p(planes.data_ptr()), B, self.depth, n,
                                          ctypes.c_void_p(self.w1.data_ptr()), ctypes.c_void_p(self.b1.data_ptr()),
                                          ctypes.c_void_p(self.w2.data_ptr()), ctypes.c_void_p(self.b2.data_ptr()),
                                          C, ctypes.c_void_p(y.data_ptr()), C, wp, work.numel(), tp,
                                          tickets.numel() - 1, st))
            x, strides, H, cin, first = y, (n * n * C, n * C, C, 1), n, C, 3
        for i, pad in enumerate(self.pads, start=1):
            if i < first:
                continue
            Ho = H + 2 * pad - 2
            y = torch.empty((B * Ho * Ho, C), device=dev, dtype=torch.float32)
            _lib.check(L.azg_small_conv3x3(ctypes.c_void_p(x.data_ptr()), *strides, B, H, pad,
                                           ctypes.c_void_p(getattr(self, f"w{i}").data_ptr()), cin, C,
                                           ctypes.c_void_p(getattr(self, f"b{i}").data_ptr()), 1,
                                           ctypes.c_void_p(y.data_ptr()), C, wp, work.numel(), tp,
                                           tickets.numel() - 1, st))
            x, H, cin = y, Ho, C
            strides = (H * H * C, H * C, C, 1)
        return x, H

    def _small_ok(self, planes):
        """Whether the small-batch kernels take this forward: at most SMALL_MAX_B leaves and
        every precondition azg_small.hip's entry points check (the 3x3 layers: pad <= 1, a side
        <= 16 with <= 256 output pixels, an even channel count; the FC layers and the heads:
        K % 4 == 0 and row strides % 4 == 0, at most 1023 actions).  Any other shape takes the
        library / Winograd path instead of an AZG_ERR_ARG."""
        if not (self.small_path and planes.is_cuda and planes.shape[0] <= SMALL_MAX_B):
            return False
        C, A, n = self.w1.shape[0], self.fw3.shape[0], self.n
        h = n
        for pad in self.pads:
            if pad > 1 or h > 16 or (h + 2 * pad - 2) ** 2 > 256 or h + 2 * pad - 2 <= 0:
                return False
            h = h + 2 * pad - 2
        return (C % 2 == 0 and A <= 1023 and (h * h * C) % 4 == 0 and self.fw1.shape[1] == h * h * C
                and self.fw2.shape[1] % 4 == 0 and self.fw34.shape[1] % 4 == 0)

    def forward(self, s):
        planes = s.view(-1, self.depth, self.n, self.n)
        # the small-batch kernels whenever they apply -- for every conv form, conv="miopen" included
        if self._small_ok(planes):
            return self._forward_small(planes)
        x = planes
        hook = self.conv_hook
        fused = x.is_cuda
        impls = []
        for i in range(1, 5):
            impl = self.conv_impl if i > 1 else "miopen"
            if impl == "winograd" and x.shape[0] < WINOGRAD_MIN_BATCH:
                impl = "miopen"  # a few leaves: the 16 small GEMMs lose to one direct conv
            impls.append(impl)
        pending = None  # bias of the previous conv, to be applied (with ReLU) by this one's input transform
        carried = False  # this layer's V was written by the previous layer's fused transform
        B, H = x.shape[0], self.n
        first_fused = (fused and self.fuse_transforms and impls[1] == "winograd" and self.pads == [1, 1, 0, 0]
                       and self.depth <= 4 and 3 <= self.n <= 9 and self.w1c.shape[0] % 64 == 0)
        if not first_fused:  # the fused front end reads the NCHW planes as they are
            x = planes.contiguous(memory_format=torch.channels_last)
        for i, pad in enumerate(self.pads, start=1):
            impl = impls[i - 1]
            h_out = H + 2 * pad - 2
            fuse_next = (fused and self.fuse_transforms and impl == "winograd" and i < 4
                         and impls[i] == "winograd" and self.pads[i] == 0)
            if fused and impl == "auto":
                impl = self._pick(x, i, pad)
            if hook:
                hook(i, "start")
            if i == 1 and first_fused:
                self._first_winograd(planes.contiguous())
                carried = True
            elif not fused:
                x = torch.relu_(F.conv2d(x, getattr(self, f"w{i}"), getattr(self, f"b{i}"), padding=pad))
            elif impl == "azg":
                x = self._conv_azg(x, i, pad)
            elif impl == "winograd":
                split_out = i == 4 and self.fc1_split and self.gemm != "f32" and (
                    B >= FC1_SPLIT_MIN_BATCH or (self.fc_tail_small and B % 256 == 0))
                x = self._conv_winograd(x, i, pad, in_bias=pending, carried=carried, B=B, H=H, fuse_next=fuse_next,
                                        split_out=split_out)
                if split_out:
                    x = ("split", x)
                pending = None
                carried = fuse_next
            elif i == 1 and impls[1] == "winograd":
                # conv1's bias + ReLU ride in conv2's Winograd input transform (no separate pass)
                x = F.conv2d(x, self.w1, None, padding=pad)
                pending = self.b1
            else:
                x = self._conv_miopen(x, i, pad)
            if hook:
                hook(i, "stop")
            H = h_out
        if isinstance(x, tuple):
            return self._fc_split(x[1])
        else:
            x = x.permute(0, 2, 3, 1).reshape(x.shape[0], -1)  # NHWC flatten, no copy
            # f32 FC tail (small batches): bias + ReLU in the GEMMs' epilogue
            x = _addmm_relu(self.fb1, x, self.fw1.t())
        x = _addmm_relu(self.fb2, x, self.fw2.t())
        A = self.fw3.shape[0]
        if x.is_cuda and A <= 1024:  # [fc3 | fc4] then P, v in one libazg kernel (azg_policy_value)
            import ctypes
            from . import _lib
            pv = torch.mm(x, self.fw34.t())  # [B, A + 1]; the bias is added by the kernel
            p = torch.empty((x.shape[0], A), device=x.device, dtype=torch.float32)
            v = torch.empty((x.shape[0], 1), device=x.device, dtype=torch.float32)
            _lib.check(_lib.lib().azg_policy_value(
                ctypes.c_void_p(pv.data_ptr()), A + 1, ctypes.c_void_p(self.fb34.data_ptr()), 1.0,
                ctypes.c_void_p(p.data_ptr()), ctypes.c_void_p(v.data_ptr()), x.shape[0], A,
                ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream)))
            return p, v
        pv = torch.addmm(self.fb34, x, self.fw34.t())  # [B, A + 1]: fc3 logits | fc4
        return torch.exp(torch.log_softmax(pv[:, :A], dim=1)), torch.tanh(pv[:, A:])  # NNet.py:94


def replay_form(net):
    """The evaluator self-play and the arena fall back to when the split-fp16 form
    meets an operand fp16 cannot hold (InferenceNet.check_range): direct f32
    convolutions (MIOpen; per-layer error ~6.5e-7 relative, profiles/r02_wino_layer_error.json)
    and the f32 FC tail, not the f32-GEMM Winograd form, whose F(5,3)/F(4,3) tiles
    carry the largest error of the three (1.6e-5 at conv3) -- the fallback runs for
    exactly the large-activation networks where that would matter."""
    return InferenceNet(net, conv="miopen", gemm="f32")


class NNetWrapper:
    """Reference NNetWrapper surface (NNet.py:27-120) over InflexionNNet."""

    _tuned_read = None  # whether TunableOp accepted TUNABLEOP_RESULTS (read once per process)

    def __init__(self, game=None, args=None, device=None):
        a = dict(DEFAULT_ARGS)
        a.update(args or {})
        self.args = a
        if game is not None:
            depth, bx, by = game.to_planes().shape
            action_size = game.max_actions
        else:
            depth, bx, action_size = 4, 7, 343
        self.depth, self.board_x, self.board_y, self.action_size = depth, bx, bx, action_size
        self.nnet = InflexionNNet(bx, depth, action_size, a["num_channels"], a["dropout"])
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu"))
        self.nnet.to(self.device)

    def predict(self, board):
        """Batch-1 predict (NNet.py:78-94): planes -> (P f32[A], v f32[1])."""
        x = torch.as_tensor(np.asarray(board).astype(np.float64), dtype=torch.float32, device=self.device)
        x = x.view(self.depth, self.board_x, self.board_y)
        self.nnet.eval()
        with torch.no_grad():
            pi, v = self.nnet(x)
        return torch.exp(pi).cpu().numpy()[0], v.cpu().numpy()[0]

    def predict_batch(self, planes):
        self.nnet.eval()
        with torch.no_grad():
            pi, v = self.nnet(planes)
        return torch.exp(pi), v.view(-1)

    def _train_forward(self, x):
        """The training forward: InflexionNNet.forward, with conv2-4 on libazg's training
        kernels (wino_train.train_forward) on the GPU in f32 when args["train_conv"] is
        "winograd" -- the module itself otherwise (CPU: the reference's arithmetic)."""
        if x.is_cuda and self.args.get("train_conv", "winograd") == "winograd" and self.args["train_dtype"] == "f32":
            from .wino_train import applies_net, train_forward
            if applies_net(self.nnet, x):
                return train_forward(self.nnet, x)
        return self.nnet(x)

    def _train_losses(self, x, tp, tv):
        """(l_pi, l_v) of a training step (NNet.py:57-61, 96-100).  On the Winograd training path the
        heads and both losses run on libazg (wino_train.train_losses: 3 launches, args["fused_loss"],
        default on); otherwise the reference's torch expressions on _train_forward's outputs."""
        if (self.args.get("fused_loss", True) and x.is_cuda and self.args.get("train_conv", "winograd") == "winograd"
                and self.args["train_dtype"] == "f32"):
            from .wino_train import applies_net, train_losses
            if applies_net(self.nnet, x):
                return train_losses(self.nnet, x, tp, tv)
        out_pi, out_v = self._train_forward(x)
        l_pi = -torch.sum(tp * out_pi) / tp.size()[0]
        l_v = torch.sum((tv - out_v.view(-1)) ** 2) / tv.size()[0]
        return l_pi, l_v

    def _adam(self):
        """torch.optim.Adam() as NNet.py:37 builds it.  On the GPU: args["optimizer"] "azg" (default)
        is optim.FusedAdam, the capturable foreach form's arithmetic in one libazg launch per step;
        "torch" is torch's own capturable form (step count and bias corrections on the device) --
        either way the form _train_graph replays, so the eager and the graph-replayed trainer take
        the same update.  The CPU keeps the reference's exact Adam."""
        if (self.device.type == "cuda" and self.args.get("optimizer", "azg") == "azg"
                and not self.args["fused_adam"]):
            from .optim import FusedAdam
            return FusedAdam(self.nnet.parameters())
        kw = {"capturable": True} if self.device.type == "cuda" else {}
        if self.args["fused_adam"]:
            kw["fused"] = True
        return torch.optim.Adam(self.nnet.parameters(), **kw)

    def _autocast(self, cache=True):
        dt = self.args["train_dtype"]
        if dt not in ("f32", "bf16"):
            raise ValueError(f"train_dtype must be 'f32' or 'bf16', got {dt!r}")
        return torch.autocast(self.device.type, dtype=torch.bfloat16, enabled=dt == "bf16", cache_enabled=cache)

    def train(self, examples):
        """Reference training loop (NNet.py:36-76): Adam, 10 epochs of batches
        sampled with replacement from numpy's global RNG (examples as the reference's list of
        (planes, pi, v)); on the GPU with train_examples' out-of-range rule (_overflow_replay)."""
        return self._overflow_replay(lambda: self._train_list(examples))

    def _train_list(self, examples):
        opt = self._adam()
        bs = self.args["batch_size"]
        for _ in range(self.args["epochs"]):
            self.nnet.train()
            for _ in range(int(len(examples) / bs)):
                ids = np.random.randint(len(examples), size=bs)
                boards, pis, vs = list(zip(*[examples[i] for i in ids]))
                boards = torch.FloatTensor(np.array(boards).astype(np.float64)).to(self.device)
                tp = torch.FloatTensor(np.array(pis)).to(self.device)
                tv = torch.FloatTensor(np.array(vs).astype(np.float64)).to(self.device)
                with self._autocast():
                    out_pi, out_v = self._train_forward(boards)
                    l_pi = -torch.sum(tp * out_pi) / tp.size()[0]
                    l_v = torch.sum((tv - out_v.view(-1)) ** 2) / tv.size()[0]
                opt.zero_grad()
                (l_pi + l_v).backward()
                opt.step()

    def train_examples(self, ex, group=None, stats=None):
        """NNet.py:36-76 on an ExampleSet already resident on the device: the same
        Adam, epochs and batch draws (np.random.randint on numpy's global stream,
        so the sampled batches are the reference's), with the batch gathered on
        the GPU instead of converted from Python lists.  Returns per-batch
        (l_pi, l_v) as a device tensor [batches, 2].

        On the GPU the steps after the first _GRAPH_EAGER_STEPS replay one captured HIP
        graph of the whole step (args["train_graph"], default on: _train_graph).  When the
        Winograd training convolutions (wino_train) met an operand fp16 cannot hold, the
        call is undone -- weights, BatchNorm buffers, numpy's and torch's RNG states -- and
        run again with the library convolutions (the self-play replay_form rule applied to
        training), so the result never carries a saturated operand.

        group: a torch.distributed group of more than one rank trains data-parallel
        (ddp.train_examples_dp: each batch split over the ranks, whole-batch
        BatchNorm statistics, one gradient all-reduce per step); every rank of the
        group calls this with the same examples.  stats: a dict that receives the step
        count (and, data-parallel, the collectives' accounting)."""
        dp = None
        if group is not None:
            import torch.distributed as dist
            if dist.get_world_size(group) > 1:
                from .ddp import train_examples_dp
                dp = dist

        def run():
            if dp is not None:
                return train_examples_dp(self, ex, group, stats=stats)
            return self._train_single(ex, stats)

        with self._tuned_gemms():
            losses = self._overflow_replay(run, group if dp is not None else None)
        if stats is not None and self.last_replayed_library:
            stats["replayed_library"] = True
        return losses

    @contextlib.contextmanager
    def _tuned_gemms(self):
        """The trainer's library GEMMs (the FC layers on hipBLASLt, f32) under torch's TunableOp for the
        call, each GEMM shape on its fastest hipBLASLt / rocBLAS solution (+3% examples/s at batch 512,
        profiles/r06_train_tunableop.json).  The solutions come from TUNABLEOP_RESULTS (tuned once by
        tools/tune_gemms.py); when that file is absent or TunableOp rejects it (another torch, ROCm or
        GPU), or args["tunable_gemm"] is "tune", each shape is measured once per process instead, in the
        eager steps before the step is captured (a few seconds on a process's first call).
        args["tunable_gemm"] False keeps the heuristic's choice.  The process-wide TunableOp switches are
        restored afterwards."""
        mode = self.args.get("tunable_gemm", True)
        on = self.device.type == "cuda" and bool(mode) and hasattr(torch.cuda, "tunable")
        if not on:
            yield
            return
        tun = torch.cuda.tunable
        prev = (tun.is_enabled(), tun.tuning_is_enabled())
        if not prev[0]:  # (a user's own TunableOp settings are left as they are)
            import tempfile
            tun.set_filename(os.path.join(tempfile.gettempdir(), f"azg_tunableop_{os.getpid()}.csv"))
        tun.enable(True)
        tuned = False
        if mode != "tune" and os.path.exists(TUNABLEOP_RESULTS):
            if NNetWrapper._tuned_read is None:
                NNetWrapper._tuned_read = bool(tun.read_file(TUNABLEOP_RESULTS))
            tuned = NNetWrapper._tuned_read
        tun.tuning_enable(not tuned)
        tun.set_max_tuning_duration(30)  # ms per GEMM shape
        try:
            yield
        finally:
            tun.tuning_enable(prev[1])
            tun.enable(prev[0])

    def _overflow_replay(self, run, group=None):
        """run() (a training call); if the Winograd training convolutions met an operand fp16
        cannot hold, undo it -- weights, BatchNorm buffers, numpy's and torch's streams -- and
        run it again on the library convolutions (every rank of `group` when one saw it)."""
        self.last_replayed_library = False
        dp = None
        if group is not None:
            import torch.distributed as dp
        wino = (self.device.type == "cuda" and self.args.get("train_conv", "winograd") == "winograd"
                and self.args["train_dtype"] == "f32")
        if not wino:
            return run()
        from . import wino_train
        wino_train.take_flag(self.device)  # a stale flag from an earlier call is not this call's
        saved = ({k: v.detach().clone() for k, v in self.nnet.state_dict().items()}, np.random.get_state(),
                 torch.get_rng_state(), torch.cuda.get_rng_state(self.device))
        losses = run()
        flag = wino_train.take_flag(self.device)
        if dp is not None:  # every rank replays when any rank saw an out-of-range operand
            backend_dev = self.device if dp.get_backend(group) == "nccl" else torch.device("cpu")
            t = torch.tensor([flag], dtype=torch.int32, device=backend_dev)
            dp.all_reduce(t, op=dp.ReduceOp.MAX, group=group)
            flag = int(t.item())
        if flag:
            sd, nps, cpu_rng, dev_rng = saved
            self.nnet.load_state_dict(sd)
            np.random.set_state(nps)
            torch.set_rng_state(cpu_rng)
            torch.cuda.set_rng_state(dev_rng, self.device)
            conv = self.args["train_conv"]
            self.args["train_conv"] = "library"
            try:
                losses = run()
            finally:
                self.args["train_conv"] = conv
            self.last_replayed_library = True
        return losses

    def _train_single(self, ex, stats):
        bs = self.args["batch_size"]
        E = len(ex)
        nb = int(E / bs)
        losses = torch.zeros((self.args["epochs"] * nb, 2), dtype=torch.float32, device=self.device)
        planes = ex.planes.to(self.device)
        pis = ex.pis.to(self.device)
        vs = ex.vs.to(self.device)
        if stats is not None:
            stats["steps"] = self.args["epochs"] * nb
        if (self.args.get("train_graph", True) and self.device.type == "cuda"
                and self.args["epochs"] * nb > _GRAPH_EAGER_STEPS):
            if stats is not None:
                stats["graph"] = True
            self._train_graph(planes, pis, vs, nb, losses)
            return losses
        opt = self._adam()
        k = 0
        for _ in range(self.args["epochs"]):
            self.nnet.train()
            # the epoch's nb batch draws of NNet.py:52 in one call (numpy's legacy randint draws
            # element by element, so this is the same stream as nb calls of size bs) and one upload:
            # no host-device synchronisation inside the epoch
            ids_all = torch.from_numpy(np.random.randint(E, size=(nb, bs))).to(self.device) if nb else None
            for j in range(nb):
                ids = ids_all[j]
                tp, tv = pis[ids], vs[ids]
                with self._autocast():
                    l_pi, l_v = self._train_losses(planes[ids], tp, tv)
                opt.zero_grad()
                (l_pi + l_v).backward()
                opt.step()
                losses[k, 0] = l_pi.detach()
                losses[k, 1] = l_v.detach()
                k += 1
        return losses

    def _train_graph(self, planes, pis, vs, nb, losses):
        """_train_single's loop with the step replayed as one captured HIP graph: forward
        (conv2-4 on the Winograd training kernels), the losses, backward and the Adam update
        are ~400 launches per 512-example step, whose host-side issue cost the GPU more
        time than their work.  The same batches are drawn at the same points of numpy's
        stream; the first _GRAPH_EAGER_STEPS steps run eagerly on a side stream (real
        steps, which also warm up every kernel's one-time queries and the allocator), then
        one step is captured and replayed, each replay reading the batch's indices from a
        static buffer.  Adam is torch's capturable form, as in the eager GPU loop (_adam);
        dropout draws from torch's graph-safe philox offsets."""
        bs = self.args["batch_size"]
        dev = self.device
        E = planes.shape[0]
        opt = self._adam()
        # steps per captured graph: one replay runs gs whole steps (each with its own batch, forward,
        # backward and Adam update; gradients zeroed in between), so the host issues one launch per
        # gs steps; an epoch's last nb % gs steps run eagerly
        gs = max(1, int(self.args.get("train_graph_steps", TRAIN_GRAPH_STEPS)))
        gs = min(gs, max(1, nb))
        ids_buf = torch.zeros((gs, bs), dtype=torch.int64, device=dev)
        loss_buf = torch.zeros((gs, 2), dtype=torch.float32, device=dev)

        def step(i):
            tp, tv = pis[ids_buf[i]], vs[ids_buf[i]]
            with self._autocast(cache=False):
                l_pi, l_v = self._train_losses(planes[ids_buf[i]], tp, tv)
            (l_pi + l_v).backward()
            opt.step()
            loss_buf[i, 0].copy_(l_pi.detach())
            loss_buf[i, 1].copy_(l_v.detach())

        def steps():
            for i in range(gs):
                if i:
                    opt.zero_grad(set_to_none=False)  # (the captured grads exist: zero, then accumulate)
                step(i)

        cur = torch.cuda.current_stream(dev)
        side = torch.cuda.Stream(dev)
        graph = None
        eager = False  # set when the capture failed: the remaining steps run eagerly
        k = 0
        self.nnet.train()
        try:
            for _ in range(self.args["epochs"]):
                ids_all = torch.from_numpy(np.random.randint(E, size=(nb, bs))).to(dev) if nb else None
                j = 0
                while j < nb:
                    if graph is None and not eager and k >= _GRAPH_EAGER_STEPS and j + gs <= nb:
                        # capture gs steps (nothing executes during a capture; a failed one leaves the
                        # weights, the optimizer's device state and the RNG where they were)
                        try:
                            g = torch.cuda.CUDAGraph()
                            opt.zero_grad(set_to_none=True)
                            with torch.cuda.graph(g):
                                steps()
                            graph = g
                        except RuntimeError as err:
                            from ._lib import AzgError
                            if isinstance(err, AzgError):  # a libazg argument / HIP error is not a refused capture
                                raise
                            import warnings
                            warnings.warn(f"train_examples: the training step could not be captured as a HIP "
                                          f"graph ({err}); the remaining steps run eagerly")
                            eager = True
                            torch.cuda.synchronize(dev)
                    if graph is not None and j + gs <= nb:
                        ids_buf.copy_(ids_all[j:j + gs])
                        graph.replay()
                        losses[k:k + gs].copy_(loss_buf)
                        k += gs
                        j += gs
                        continue
                    side.wait_stream(cur)
                    with torch.cuda.stream(side):
                        ids_buf[0].copy_(ids_all[j])
                        opt.zero_grad(set_to_none=graph is None)
                        step(0)
                        losses[k].copy_(loss_buf[0])
                    cur.wait_stream(side)
                    k += 1
                    j += 1
        finally:
            if graph is not None:
                torch.cuda.current_stream(dev).synchronize()
                # the parameters' .grad live in the graph's pool: hand back plain tensors
                for p in self.nnet.parameters():
                    if p.grad is not None:
                        p.grad = p.grad.clone()
                del graph

    def save_checkpoint(self, folder="checkpoint", filename="checkpoint.pth.tar"):
        os.makedirs(folder, exist_ok=True)
        torch.save({"state_dict": self.nnet.state_dict()}, os.path.join(folder, filename))

    def load_checkpoint(self, folder="checkpoint", filename="checkpoint.pth.tar"):
        path = os.path.join(folder, filename)
        if not os.path.exists(path):
            raise FileNotFoundError(f"No model in path {path}")
        ck = torch.load(path, map_location=self.device, weights_only=True)
        self.nnet.load_state_dict(ck["state_dict"])
