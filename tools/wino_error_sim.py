"""CPU error model of the network's Winograd + split-fp16 forward, for choosing tile
sizes and interpolation points (no GPU needed).

Emulates InferenceNet(gemm="split") layer by layer: conv1 direct in f32, then per
Winograd layer V = B^T d B in f32, V split to fp16 hi/lo, U = G g G^T in f64 scaled and
split, M = Vh.Uh + Vl.Uh + Vh.Ul with f32 sums (products of fp16 pairs are exact in f32),
Y = A^T M A in f32, bias, ReLU; FC heads in f32.  Reports the max relative error of P
and the max abs error of v against an f64 forward of the reference module, for the
shipped tiling and for alternatives (F(4,3) with several point sets).

    python tools/wino_error_sim.py [--leaves 256]
"""
import argparse
import itertools
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def cook_toom(m, points, scale_rows=True):
    """(A^T [m][n], G [n][3], B^T [n][n]) of F(m, 3) on the finite points + inf, f64.
    B^T is solved from the bilinear identity; rows of B^T are scaled to max |entry| 1
    (the inverse scale goes into G, which is applied in f64 to the weights)."""
    r = 3
    n = m + r - 1
    p = [float(x) for x in points]
    assert len(p) == n - 1
    AT = np.zeros((m, n))
    G = np.zeros((n, r))
    for j, pj in enumerate(p):
        AT[:, j] = [pj ** i for i in range(m)]
        N = np.prod([pj - pl for l, pl in enumerate(p) if l != j])
        G[j] = [pj ** k / N for k in range(r)]
    AT[m - 1, n - 1] = 1.0
    G[n - 1, r - 1] = 1.0
    # solve sum_j AT[i,j] G[j,k] BT[j,l] = [l == i + k] for BT
    rows, rhs = [], []
    for i in range(m):
        for k in range(r):
            for l in range(n):
                row = np.zeros((n, n))
                for j in range(n):
                    row[j, l] = AT[i, j] * G[j, k]
                rows.append(row.ravel())
                rhs.append(1.0 if l == i + k else 0.0)
    sol, res, rank, _ = np.linalg.lstsq(np.array(rows), np.array(rhs), rcond=None)
    BT = sol.reshape(n, n)
    BT[np.abs(BT) < 1e-12] = 0.0
    if scale_rows == "int":  # rows of B^T scaled to small integers (exact in f32)
        from fractions import Fraction
        from math import lcm
        for j in range(n):
            den = 1
            for x in BT[j]:
                den = lcm(den, Fraction(x).limit_denominator(64).denominator)
            s = np.abs(BT[j]).max()
            BT[j] = np.round(BT[j] * den / s * s)
            G[j] /= den
    elif scale_rows:
        for j in range(n):
            s = np.abs(BT[j]).max()
            BT[j] /= s
            G[j] *= s
    # verify
    g = np.random.randn(r)
    d = np.random.randn(n)
    y = AT @ ((G @ g) * (BT @ d))
    want = np.array([sum(g[k] * d[i + k] for k in range(r)) for i in range(m)])
    assert np.allclose(y, want, atol=1e-9), (y, want)
    return AT, G, BT


def split16(x):
    hi = x.half().float()
    lo = (x - hi).half().float()
    return hi, lo


def wino_layer(x, w, b, pad, seq, mats):
    """x [B,C,H,H] f32 -> relu(conv3x3(x) + b) by Winograd tiles of output sides seq
    (a list for both axes, or a (rows, columns) pair of lists)."""
    B, C, H, _ = x.shape
    K = w.shape[0]
    xp = F.pad(x, (pad, pad, pad, pad))
    Ho = H + 2 * pad - 2
    seqr, seqc = seq if isinstance(seq, tuple) else (seq, seq)
    assert sum(seqr) == Ho and sum(seqc) == Ho
    offr = [sum(seqr[:i]) for i in range(len(seqr))]
    offc = [sum(seqc[:i]) for i in range(len(seqc))]
    y = torch.zeros((B, K, Ho, Ho), dtype=torch.float32)
    for (i, ma), (j, mb) in itertools.product(enumerate(seqr), enumerate(seqc)):
        ATa, Ga, BTa = mats[ma]
        ATb, Gb, BTb = mats[mb]
        na, nb = ma + 2, mb + 2
        d = xp[:, :, offr[i]:offr[i] + na, offc[j]:offc[j] + nb]  # [B,C,na,nb]
        BTa32 = torch.tensor(BTa, dtype=torch.float32)
        BTb32 = torch.tensor(BTb, dtype=torch.float32)
        V = torch.einsum("ar,bcrs,ts->bcat", BTa32, d, BTb32)  # f32
        U = torch.einsum("ar,kcrs,bs->abck", torch.tensor(Ga), w.double(), torch.tensor(Gb))  # f64 [na,nb,C,K]
        amax = float(U.abs().max())
        k = int(np.floor(np.log2(1024.0 / amax)))
        Us = U * 2.0 ** k
        Uh = Us.half().double()
        Ul = (Us - Uh).half().double()
        Uh, Ul = Uh.float(), Ul.float()
        Vh, Vl = split16(V)
        # [na,nb] GEMMs: M[b,a,t,k] = sum_c V[b,c,a,t] U[a,t,c,k]
        M = (torch.einsum("bcat,atck->batk", Vh, Uh) + torch.einsum("bcat,atck->batk", Vl, Uh)
             + torch.einsum("bcat,atck->batk", Vh, Ul))
        ATa32 = torch.tensor(ATa, dtype=torch.float32)
        ATb32 = torch.tensor(ATb, dtype=torch.float32)
        Y = torch.einsum("ia,batk,jt->bkij", ATa32, M, ATb32) * float(2.0 ** -k)
        y[:, :, offr[i]:offr[i] + ma, offc[j]:offc[j] + mb] = Y
    return torch.relu(y + b.view(1, -1, 1, 1))


def fold(net):
    from azg_amd.nnet import _fold_bn
    ws = []
    for i in range(1, 5):
        ws.append(_fold_bn(getattr(net, f"conv{i}").weight, getattr(net, f"conv{i}").bias, getattr(net, f"bn{i}")))
    f1 = _fold_bn(net.fc1.weight, net.fc1.bias, net.fc_bn1)
    f2 = _fold_bn(net.fc2.weight, net.fc2.bias, net.fc_bn2)
    return ws, f1, f2


def forward(net, x, seqs, mats):
    ws, f1, f2 = fold(net)
    pads = [1, 1, 0, 0]
    h = torch.relu(F.conv2d(x, ws[0][0], ws[0][1], padding=1))
    for li in range(1, 4):
        w, b = ws[li]
        h = wino_layer(h, w, b, pads[li], seqs[li - 1], mats)
    h = h.reshape(h.shape[0], -1)
    h = torch.relu(h @ f1[0].t() + f1[1])
    h = torch.relu(h @ f2[0].t() + f2[1])
    p = torch.softmax(h @ net.fc3.weight.t() + net.fc3.bias, dim=1)
    v = torch.tanh(h @ net.fc4.weight.t() + net.fc4.bias)
    return p, v


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--leaves", type=int, default=128)
    ap.add_argument("--seed", type=int, default=6)
    a = ap.parse_args()
    torch.set_num_threads(8)
    from azg_amd.nnet import InflexionNNet
    torch.manual_seed(a.seed)
    net = InflexionNNet().eval()
    x = (torch.rand(a.leaves, 4, 7, 7) < 0.3).float()
    with torch.no_grad():
        ref = InflexionNNet().eval().double()
        ref.load_state_dict(net.state_dict())
        logp, v64 = ref(x.double())
        p64 = torch.exp(logp)
        logp32, v32m = net(x)  # the f32 reference module (direct convs)
        base = {"f32 module": (((torch.exp(logp32).double() - p64).abs() / p64).max().item(),
                               (v32m.double() - v64).abs().max().item())}
        m2, m3 = cook_toom(2, [0, 1, -1]), cook_toom(3, [0, 1, -1, 2])
        m4 = cook_toom(4, [0, 1, -1, 2, -0.5], "int")
        m5 = cook_toom(5, [0, 1, -1, -0.5, -2, 1.5], "int")  # azg_winograd.hip's F(5,3)
        shipped = {2: m2, 3: m3, 4: m4, 5: m5}
        configs = {"shipped 4+3 / 5 / 3 (121 + 49 + 25 points)": (shipped, [[4, 3], [5], [3]])}
        # conv2 as one F(7,3) tile (81 points) or F(6,3) + F(1,3)... : candidate point sets
        for pts in ([0, 1, -1, 2, -2, 0.5, -0.5, 1.5], [0, 1, -1, 2, -2, 0.5, -0.5, -1.5],
                    [0, 1, -1, 2, -0.5, 0.5, -2, 3], [0, 1, -1, 0.5, -0.5, 2, -2, 0.25],
                    [0, 1, -1, 2, -2, 0.5, -0.5, 4], [0, 1, -1, 1.5, -1.5, 0.5, -0.5, 2]):
            try:
                m7 = cook_toom(7, pts, "int")
            except AssertionError:
                continue
            mats = dict(shipped)
            mats[7] = m7
            configs[f"7 (F(7,3) pts {pts}) / 5 / 3"] = (mats, [[7], [5], [3]])
            configs[f"7 x 4+3 (99 points) / 5 / 3, pts {pts}"] = (mats, [([7], [4, 3]), [5], [3]])
        for pts in ([0, 1, -1, 2, -2, 0.5, -0.5], [0, 1, -1, 2, -0.5, 0.5, -2]):
            m6 = cook_toom(6, pts, "int")
            mats = dict(shipped)
            mats[6] = m6
            configs[f"6+1? no: F(6,3) pts {pts} as 7 = 6+1 skipped"] = None
        for name, cfg in configs.items():
            if cfg is None:
                continue
            mats, seqs = cfg
            p, v = forward(net, x, seqs, mats)
            base[name] = (((p.double() - p64).abs() / p64).max().item(), (v.double() - v64).abs().max().item())
    for k, (ep, ev) in base.items():
        print(f"{k:45s} P max rel {ep:.3e}   v max abs {ev:.3e}")


if __name__ == "__main__":
    main()
