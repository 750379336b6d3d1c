"""ctypes binding of the CPU oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE: imported only by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py -- never by the product package.
"""
import ctypes
import gzip
import json
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "liboracle.so")
GOLDEN = os.path.join(ROOT, "tests", "golden")

EVAL_FN = ctypes.CFUNCTYPE(None, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float),
                           ctypes.POINTER(ctypes.c_float), ctypes.c_void_p)

_lib = None


def build():
    src = os.path.join(ORACLE_DIR, "oracle.c")
    if not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.POINTER
        L.orc_rng_seed.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
        L.orc_rng_u32.argtypes = [ctypes.c_void_p]
        L.orc_rng_u32.restype = ctypes.c_uint32
        L.orc_rng_randint.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64]
        L.orc_rng_randint.restype = ctypes.c_int64
        L.orc_rng_random_sample.argtypes = [ctypes.c_void_p]
        L.orc_rng_random_sample.restype = ctypes.c_double
        L.orc_rng_choice_p.argtypes = [ctypes.c_void_p, P(ctypes.c_double), ctypes.c_int]
        L.orc_rng_choice_p.restype = ctypes.c_int
        L.orc_pairwise_sum_f32.argtypes = [P(ctypes.c_float), ctypes.c_int]
        L.orc_pairwise_sum_f32.restype = ctypes.c_float
        L.orc_sym_gather.argtypes = [ctypes.c_int] * 4 + [P(ctypes.c_int)]
        L.orc_stub_eval.argtypes = [P(ctypes.c_int32), ctypes.c_int, P(ctypes.c_float), P(ctypes.c_float)]
        L.orc_episode.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_int,
                                  ctypes.c_uint32, EVAL_FN, ctypes.c_void_p,
                                  P(ctypes.c_int32), P(ctypes.c_int32), P(ctypes.c_int8), ctypes.c_int,
                                  P(ctypes.c_int64)]
        L.orc_episode.restype = ctypes.c_int
        L.orc_episode_kind.argtypes = [ctypes.c_int] + L.orc_episode.argtypes
        L.orc_episode_kind.restype = ctypes.c_int
        L.orc_othello_init.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.orc_dihedral_gather.argtypes = [ctypes.c_int, ctypes.c_int, P(ctypes.c_int)]
        L.orc_stub_eval_c.argtypes = [P(ctypes.c_int32), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                      P(ctypes.c_float), P(ctypes.c_float)]
        L.orc_valid_mask.argtypes = [ctypes.c_void_p, P(ctypes.c_uint8)]
        L.orc_valid_mask.restype = ctypes.c_int
        L.orc_apply.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.orc_apply.restype = ctypes.c_int
        L.orc_planes.argtypes = [ctypes.c_void_p, P(ctypes.c_int32)]
        L.orc_game_init.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        _lib = L
    return _lib


def ptr(a, ct):
    return a.ctypes.data_as(ctypes.POINTER(ct))


class Rng:
    def __init__(self, seed):
        self.buf = ctypes.create_string_buffer(624 * 4 + 8)
        lib().orc_rng_seed(self.buf, seed)

    def u32(self):
        return lib().orc_rng_u32(self.buf)

    def randint(self, lo, hi):
        return lib().orc_rng_randint(self.buf, lo, hi)

    def random_sample(self):
        return lib().orc_rng_random_sample(self.buf)

    def choice_p(self, p):
        p = np.ascontiguousarray(p, np.float64)
        return lib().orc_rng_choice_p(self.buf, ptr(p, ctypes.c_double), len(p))


class OrcGame(ctypes.Structure):
    _fields_ = [("board", ctypes.c_int8 * 64), ("n", ctypes.c_int), ("turn", ctypes.c_int),
                ("max_turns", ctypes.c_int), ("player", ctypes.c_int), ("outcome", ctypes.c_int),
                ("kind", ctypes.c_int)]


INFLEXION, OTHELLO = 1, 2


OUTCOME_VALUE = {0: 0.0, 1: 1e-4, 2: 1.0, 3: -1.0}


def sym_gather(n, k, shift, axis):
    src = np.zeros(n * n, np.int32)
    lib().orc_sym_gather(n, k, shift, axis, ptr(src, ctypes.c_int))
    return src


def stub_eval(planes, n=7):
    planes = np.ascontiguousarray(planes, np.int32).reshape(-1)
    P = np.zeros(7 * n * n, np.float32)
    v = np.zeros(1, np.float32)
    lib().orc_stub_eval(ptr(planes, ctypes.c_int32), n, ptr(P, ctypes.c_float), ptr(v, ctypes.c_float))
    return P, v


def episode(n=7, max_turns=343, sims=25, cpuct=1.0, temp_threshold=30, seed=0, evaluator=None,
            max_moves=400, kind=INFLEXION):
    """Run one oracle episode.  evaluator(planes f32[C,n,n]) -> (P f32[A], v float)."""
    A = 7 * n * n if kind == INFLEXION else n * n + 1
    C = 4 if kind == INFLEXION else 2
    actions = np.zeros(max_moves, np.int32)
    counts = np.zeros((max_moves, A), np.int32)
    temps = np.zeros(max_moves, np.int8)
    stats = np.zeros(16, np.int64)
    cb = EVAL_FN()
    if evaluator is not None:
        def _cb(planes_p, P_p, v_p, _user):
            planes = np.ctypeslib.as_array(planes_p, shape=(C, n, n))
            P, v = evaluator(planes)
            np.ctypeslib.as_array(P_p, shape=(A,))[:] = P
            v_p[0] = float(v)
        cb = EVAL_FN(_cb)
    moves = lib().orc_episode_kind(kind, n, max_turns, sims, float(cpuct), temp_threshold, seed, cb, None,
                              ptr(actions, ctypes.c_int32), ptr(counts, ctypes.c_int32),
                              ptr(temps, ctypes.c_int8), max_moves, ptr(stats, ctypes.c_int64))
    m = min(moves, max_moves)
    return {"moves": moves, "actions": actions[:m], "counts": counts[:m], "temps": temps[:m],
            "expansions": int(stats[1]), "nodes": int(stats[2]), "final_outcome": int(stats[3]),
            "final_player": int(stats[4]), "rng_pos": int(stats[5]),
            "rng_next": [int(x) for x in stats[6:10]], "terminal_hits": int(stats[10]),
            "max_depth": int(stats[11]), "fallbacks": int(stats[12])}


def load_json(name):
    with gzip.open(os.path.join(GOLDEN, name), "rt") as f:
        return json.load(f)


def golden_counts(move, A=343):
    c = np.zeros(A, np.int32)
    for a, k in move["counts"]:
        c[a] = k
    return c


def peaked_net(module):
    """tests/golden/trained_net.npz with fc3's weight and bias times peaked_net.json.gz's fc3_scale (a
    power of two: exact) -- the peaked-prior network of make_golden.py peaked_net; returns the module."""
    import torch
    trained_net(module)
    scale = float(load_json("peaked_net.json.gz")["fc3_scale"])
    with torch.no_grad():
        module.fc3.weight.mul_(scale)
        module.fc3.bias.mul_(scale)
    return module


def golden_net(module, name):
    """The network a fixture set was recorded with: `trained*` sets trained_net, `peaked*` sets
    peaked_net, the others the manual_seed(0) module as it is."""
    if name.startswith("peaked"):
        return peaked_net(module)
    if name.startswith("trained"):
        return trained_net(module)
    return module


def trained_net(module):
    """Load tests/golden/trained_net.npz (the network the reference trains on its own self-play,
    make_golden.py trained_net) into an InflexionNNet; returns the module."""
    import torch
    d = np.load(os.path.join(GOLDEN, "trained_net.npz"))
    sd = {k[3:].replace("__", "."): torch.from_numpy(d[k].copy()) for k in d.files if k.startswith("sd_")}
    module.load_state_dict(sd)
    return module
