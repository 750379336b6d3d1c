"""ctypes binding of libazg.so (the C ABI declared in include/azg.h).

The HIP path is the only path: if the library is missing or a call fails, this
module raises -- there is no CPU fallback.  torch is imported first so that the
library binds the HIP runtime torch already loaded (same SONAME), which makes
torch tensors' device pointers and streams directly usable by the engine.
"""
import ctypes
import os
import subprocess

import torch  # noqa: F401  (load torch's libamdhip64 first)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libazg.so")
CSRC = os.path.join(HERE, "csrc")

GAME_INFLEXION = 1
GAME_OTHELLO = 2
FLAG_GC = 1
FLAG_RECORD = 2
FLAG_ARENA = 4
OPPONENT_RANDOM = 1
OPPONENT_GREEDY = 2

ERR = {0: "ok", -1: "bad argument", -2: "HIP error", -3: "node pool full", -4: "path too deep",
       -5: "no valid action", -6: "bad call order"}


ERR_NODE_POOL = -3
ERR_PATH = -4


class AzgError(RuntimeError):
    """A libazg call failed; `code` is its AZG_ERR_* value (None for errors raised in Python)."""

    def __init__(self, msg, code=None):
        super().__init__(msg)
        self.code = code


class Config(ctypes.Structure):
    _fields_ = [("game_kind", ctypes.c_int32), ("n", ctypes.c_int32), ("max_turns", ctypes.c_int32),
                ("num_games", ctypes.c_int32), ("sims", ctypes.c_int32), ("temp_threshold", ctypes.c_int32),
                ("cpuct", ctypes.c_double), ("seed_base", ctypes.c_uint32), ("pad0", ctypes.c_int32),
                ("first_game", ctypes.c_int64), ("node_capacity", ctypes.c_int32),
                ("max_depth", ctypes.c_int32), ("max_moves", ctypes.c_int32), ("flags", ctypes.c_int32)]


assert ctypes.sizeof(Config) == 64

# (name, restype, argtypes) of every symbol include/azg.h declares
_VP, _I32, _I64, _U32 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint32
SIGNATURES = [
    ("azg_create", ctypes.c_int, [ctypes.POINTER(Config), _VP, ctypes.POINTER(_VP)]),
    ("azg_destroy", None, [_VP]),
    ("azg_last_error", ctypes.c_char_p, []),
    ("azg_abi_version", ctypes.c_int, []),
    ("azg_reset", ctypes.c_int, [_VP, _U32, _I64, _VP]),
    ("azg_sim_begin", ctypes.c_int, [_VP, _VP, _VP]),
    ("azg_sim_end", ctypes.c_int, [_VP, _VP, _I32, _VP, _VP]),
    ("azg_sim_end_begin", ctypes.c_int, [_VP, _VP, _I32, _VP, _VP, _VP]),
    ("azg_stub_eval", ctypes.c_int, [_VP, _VP, _VP, _VP, _VP]),
    ("azg_move_end", ctypes.c_int, [_VP, _VP]),
    ("azg_refill", ctypes.c_int, [_VP, _VP, _I64, _U32, _VP, _I64, _VP, _VP, _VP, _VP, _VP, _VP]),
    ("azg_active_games", ctypes.c_int, [_VP, ctypes.POINTER(_I32), _VP]),
    ("azg_get_state", ctypes.c_int, [_VP, _VP, _VP, _VP, _VP, _VP, _VP]),
    ("azg_set_root", ctypes.c_int, [_VP, _I32, _VP, _I32, _I32, _VP]),
    ("azg_get_rng", ctypes.c_int, [_VP, _I32, _VP, ctypes.POINTER(_I32), _VP]),
    ("azg_set_rng", ctypes.c_int, [_VP, _I32, _VP, _I32, _VP]),
    ("azg_slot_begin", ctypes.c_int, [_VP, _I32, _VP, _I32, _I32, _VP, _I32, _VP]),
    ("azg_slot_end", ctypes.c_int, [_VP, _I32, _VP, _VP, _VP, _VP, _VP]),
    ("azg_root_counts", ctypes.c_int, [_VP, _I32, _VP, _VP]),
    ("azg_read_moves", ctypes.c_int, [_VP, _VP, _VP, _VP, _VP, _VP]),
    ("azg_stats", ctypes.c_int, [_VP, _VP, _VP]),
    ("azg_device_ptrs", ctypes.c_int, [_VP, _VP]),
    ("azg_bias_relu_nhwc", ctypes.c_int, [_VP, _VP, _I64, _I32, _VP]),
    ("azg_conv3x3_bias_relu_nhwc", ctypes.c_int, [_VP, _VP, _VP, _VP, _I32, _I32, _I32, _I32, _I32, _VP]),
    ("azg_conv3x3_variant", ctypes.c_int, [ctypes.c_int, _VP, _VP, _VP, _VP, _I32, _I32, _I32, _I32, _I32, _VP]),
    ("azg_game_info", ctypes.c_int, [_I32, _I32, _VP]),
    ("azg_winograd_layout", ctypes.c_int, [_I32, _VP, _VP]),
    ("azg_winograd_tables", ctypes.c_int, [_I32, _VP, _VP]),
    ("azg_winograd_in_nhwc", ctypes.c_int, [_VP, _VP, _VP, _I32, _I32, _I32, _I32, _I32, _VP, _VP]),
    ("azg_winograd_out_nhwc", ctypes.c_int, [_VP, _VP, _VP, _I32, _I32, _I32, _I32, ctypes.c_float, _VP]),
    ("azg_winograd_out_split", ctypes.c_int,
     [_VP, _VP, _VP, _I32, _I32, _I32, _I32, ctypes.c_float, _I32, _I32, _VP, _VP]),
    ("azg_winograd_mid_nhwc", ctypes.c_int, [_VP, _VP, _VP, _I32, _I32, _I32, ctypes.c_float, _I32, _VP, _VP]),
    ("azg_winograd_first_nchw", ctypes.c_int, [_VP, _VP, _VP, _VP, _I32, _I32, _I32, _I32, _I32, _VP, _VP]),
    ("azg_split_gemm", ctypes.c_int, [_VP, _VP, _VP, _I32, _VP, _VP, _I32, _I32, _VP]),
    ("azg_fc_act_split", ctypes.c_int, [_VP, _I32, _I64, _VP, ctypes.c_float, _VP, _I32, _I32, _I32, _VP, _VP]),
    ("azg_policy_value", ctypes.c_int, [_VP, _I32, _VP, ctypes.c_float, _VP, _VP, _I32, _I32, _VP]),
    ("azg_fc_act", ctypes.c_int, [_VP, _I32, _I64, _VP, ctypes.c_float, _VP, _I32, _I32, _I32, _I32, _I32, _VP, _VP]),
    ("azg_policy_value_parts", ctypes.c_int, [_VP, _I32, _I64, _I32, _VP, ctypes.c_float, _VP, _VP, _I32, _I32,
                                              _VP]),
    ("azg_split_gemm_variant", ctypes.c_int, [_I32, _VP, _VP, _VP, _I32, _VP, _VP, _I32, _I32, _VP]),
    ("azg_small_conv3x3", ctypes.c_int, [_VP, _I64, _I32, _I32, _I32, _I32, _I32, _I32, _VP, _I32, _I32, _VP, _I32,
                                         _VP, _I32, _VP, _I64, _VP, _I32, _VP]),
    ("azg_small_fc", ctypes.c_int, [_VP, _I32, _I32, _VP, _I32, _I32, _VP, _I32, _VP, _I32, _VP]),
    ("azg_small_conv12", ctypes.c_int, [_VP, _I32, _I32, _I32, _VP, _VP, _VP, _VP, _I32, _VP, _I32, _VP, _I64, _VP,
                                        _I32, _VP]),
    ("azg_small_heads", ctypes.c_int, [_VP, _I32, _I32, _VP, _I32, _I32, _VP, _VP, _VP, _VP, _VP, _VP]),
    ("azg_split_gemm_pick", ctypes.c_int, [_I32, _VP, _VP, _I32]),
    ("azg_set_gemm_blocks", ctypes.c_int, [_I32]),
    ("azg_set_arena", ctypes.c_int, [_VP, _VP, _VP, _VP]),
    ("azg_opponent_move", ctypes.c_int, [_VP, _I32, _VP]),
    ("azg_arena_follow", ctypes.c_int, [_VP, _VP, _VP]),
    ("azg_examples", ctypes.c_int, [_I32, _I32, _I32, _I32, _I32, _I32, _VP, _VP, _VP, _I32, _I32, _I64, _VP, _VP,
                                    _VP, ctypes.POINTER(_I64), _VP]),
    ("azg_fc_act_t", ctypes.c_int, [_VP, _I32, _I64, _VP, ctypes.c_float, _VP, _I32, _I32, _I32, _I32, _VP, _VP]),
    ("azg_absmax", ctypes.c_int, [_VP, _I64, _VP, _VP]),
    ("azg_bn_relu_fwd", ctypes.c_int, [_VP, _I64, _I32, _VP, _VP, ctypes.c_float, ctypes.c_float, _VP, _VP, _VP,
                                       _VP, _VP, _VP]),
    ("azg_bn_relu_bwd", ctypes.c_int, [_VP, _VP, _I64, _I32, _VP, _VP, _VP, _VP, _VP, _VP, _VP]),
    ("azg_bn_sums", ctypes.c_int, [_VP, _I64, _I32, _VP, _VP, _VP]),
    ("azg_bn_relu_fwd_from_sums", ctypes.c_int, [_VP, _I64, _I32, _VP, _I64, _VP, _VP, ctypes.c_float,
                                                 ctypes.c_float, _VP, _VP, _VP, _VP, _VP]),
    ("azg_bn_relu_bwd_sums", ctypes.c_int, [_VP, _VP, _I64, _I32, _VP, _VP, _VP, _VP]),
    ("azg_bn_relu_bwd_from_sums", ctypes.c_int, [_VP, _VP, _I64, _I32, _VP, _VP, _I64, _VP, _VP, _VP, _VP, _VP]),
    ("azg_conv1_train_fwd", ctypes.c_int, [_VP, _I64, _I32, _I32, _VP, _VP, _I32, _VP, _VP]),
    ("azg_conv1_train_wgrad", ctypes.c_int, [_VP, _VP, _I64, _I32, _I32, _I32, _VP, _VP, _VP, _VP]),
    ("azg_wt_u_build", ctypes.c_int, [_VP, _I32, _I32, _I32, _VP, _VP, _VP, _VP, _VP]),
    ("azg_wt_out", ctypes.c_int, [_VP, _VP, _VP, _I32, _I32, _I32, _VP, _VP]),
    ("azg_wt_dout", ctypes.c_int, [_VP, _VP, _I32, _I32, _I32, _VP, _VP, _VP]),
    ("azg_wt_din", ctypes.c_int, [_VP, _VP, _I32, _I32, _I32, _I32, _VP, _VP, _VP]),
    ("azg_wt_split2_transpose", ctypes.c_int, [_VP, _VP, _I32, _I32, _I32, _VP]),
    ("azg_wt_pow2_scale", ctypes.c_int, [_VP, ctypes.c_float, _VP, _VP]),
    ("azg_wt_dw", ctypes.c_int, [_VP, _I32, _I32, _I32, _VP, _VP, _VP]),
    ("azg_wt_dy_stats", ctypes.c_int, [_VP, _I64, _I32, _VP, _VP, _VP, _VP]),
    ("azg_examples_rows", ctypes.c_int, [_I32, _I32, _I32, _I32, _I32, _I32, _VP, _VP, _VP, _I32, _I32, _I32, _I64,
                                         _VP, _VP, _VP, ctypes.POINTER(_I64), _VP]),
    ("azg_py_shuffle", ctypes.c_int, [_VP, _I64, _VP, ctypes.POINTER(_I32)]),
    ("azg_adam_step", ctypes.c_int, [_I32, _VP, _VP, _VP, _VP, _VP, _VP, ctypes.c_double, ctypes.c_double,
                                     ctypes.c_double, ctypes.c_double, _VP]),
    ("azg_train_loss_fwd", ctypes.c_int, [_VP, _I32, _VP, _I32, _VP, _I32, _VP, _I32, _I32, _VP, _VP, _VP]),
    ("azg_train_loss_bwd", ctypes.c_int, [_VP, _I32, _VP, _I32, _VP, _I32, _VP, _VP, _I32, _I32, _VP, _VP, _I32, _VP,
                                          _I32, _VP]),
]

_lib = None


def build(force=False):
    """Compile libazg.so for gfx950 in-tree (hipcc; no GPU needed)."""
    srcs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if os.path.isfile(os.path.join(CSRC, f))]
    newest = max(os.path.getmtime(s) for s in srcs)
    if force or not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < newest:
        if force:
            subprocess.check_call(["make", "-s", "-C", CSRC, "clean"])
        subprocess.check_call(["make", "-s", "-j8", "-C", CSRC])
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise AzgError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; "
                           f"g.build()'` (no CPU fallback exists)")
        L = ctypes.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


_probes = None
PROBES_PATH = os.path.join(os.path.dirname(HERE), "tools", "libazg_probes.so")


def probes():
    """tools/libazg_probes.so: the split GEMM built with its probe-only schedules
    (azg_split_gemm_variant for every variant, azg_split_gemm_stamps).  Tools and the
    probe tests only; the product never loads it."""
    global _probes
    if _probes is None:
        if not os.path.exists(PROBES_PATH):
            subprocess.check_call(["make", "-s", "-C", os.path.dirname(PROBES_PATH)])
        L = ctypes.CDLL(PROBES_PATH)
        for name, res, args in (
                ("azg_split_gemm_variant", ctypes.c_int, [_I32, _VP, _VP, _VP, _I32, _VP, _VP, _I32, _I32, _VP]),
                ("azg_split_gemm_stamps", ctypes.c_int, [_VP, _VP, _VP, _I32, _VP, _VP, _I32, _I32, _VP, _I64, _VP]),
                ("azg_split_gemm_pick", ctypes.c_int, [_I32, _VP, _VP, _I32]),
                ("azg_split_gemm", ctypes.c_int, [_VP, _VP, _VP, _I32, _VP, _VP, _I32, _I32, _VP]),
                ("azg_last_error", ctypes.c_char_p, [])):
            if hasattr(L, name):
                fn = getattr(L, name)
                fn.restype = res
                fn.argtypes = args
        _probes = L
    return _probes


def check(rc):
    if rc != 0:
        msg = lib().azg_last_error().decode(errors="replace")
        raise AzgError(f"libazg: {ERR.get(rc, rc)} ({rc}): {msg}", rc)
    return rc
