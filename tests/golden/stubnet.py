"""Hash evaluator ("stub net") used to pin the search bit-exactly.

TEST INFRASTRUCTURE.  The real network's f32 outputs differ between CPU and GPU
in the last bits, so bit-exact parity of visit counts is pinned with a
deterministic evaluator instead: an integer hash of the (randomly symmetrised)
input planes mapped to exactly representable f32 priors and values.  The same
function is implemented three times:

  * here, in numpy (used by ``make_golden.py`` to drive the reference MCTS),
  * ``oracle/oracle.c`` ``orc_stub_eval`` (C restatement, CPU checker),
  * ``csrc/azg_kernels.hip`` ``stub_eval_kernel`` (the GPU evaluator mode).

Specification (cells indexed c = r*n + q, n*n <= 64):
    own  = sum(2**c for planes[0].flat[c] != 0)
    opp  = sum(2**c for planes[1].flat[c] != 0)
    t, k = planes[2].flat[0], planes[3].flat[0]
    h    = mix(own ^ mix(opp ^ mix((t << 1) | k)))          (splitmix64 finaliser)
    ha   = mix(h ^ ((a + 1) * 0xD1B54A32D192ED03))
    P[a] = 0 if ha >> 59 == 0 else f32(ha & 0xFFFFFF) * 2**-24
    P[:] = 0 if h >> 56 < 4          (exercises MCTS.py:100-107 fallback)
    v    = f32(((h >> 20) & 2047) - 1024) / 1024
"""
import numpy as np

M64 = (1 << 64) - 1
GOLD = 0x9E3779B97F4A7C15
A_MUL = 0xD1B54A32D192ED03


def mix(x):
    x = (x + GOLD) & M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & M64
    return x ^ (x >> 31)


def _mix_np(x):
    with np.errstate(over="ignore"):
        x = x + np.uint64(GOLD)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return x ^ (x >> np.uint64(31))


def planes_hash(planes):
    planes = np.asarray(planes)
    c0 = planes[0].ravel() != 0
    c1 = planes[1].ravel() != 0
    own = sum(1 << int(i) for i in np.nonzero(c0)[0])
    opp = sum(1 << int(i) for i in np.nonzero(c1)[0])
    t = int(planes[2].ravel()[0]) if planes.shape[0] > 2 else 0  # games with 2 planes (Othello): t = k = 0
    k = int(planes[3].ravel()[0]) if planes.shape[0] > 3 else 0
    return mix(own ^ mix(opp ^ mix(((t << 1) | k) & M64)))


def stub_eval(planes, n_actions):
    h = planes_hash(planes)
    a = np.arange(1, n_actions + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        ha = _mix_np(np.uint64(h) ^ (a * np.uint64(A_MUL)))
    p = (ha & np.uint64(0xFFFFFF)).astype(np.float32) * np.float32(2.0 ** -24)
    p[(ha >> np.uint64(59)) == 0] = np.float32(0.0)
    if (h >> 56) < 4:
        p[:] = np.float32(0.0)
    v = np.float32(((h >> 20) & 2047) - 1024) / np.float32(1024.0)
    return p.astype(np.float32), np.array([v], dtype=np.float32)
