"""C-ABI boundary checks that need no GPU: the library loads and exports every
symbol include/azg.h declares, with the declared config layout."""
import ctypes
import os
import re

import azg_amd  # noqa: F401
from azg_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "azg.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(azg_[a-z_0-9]+)\s*\(", src)))


def test_header_symbols_exported():
    L = _lib.lib()
    names = _declared()
    assert len(names) >= 18
    for n in names:
        assert hasattr(L, n), n
    assert sorted(s[0] for s in _lib.SIGNATURES) == names


def test_config_layout_and_version():
    assert ctypes.sizeof(_lib.Config) == 64
    assert _lib.Config.cpuct.offset == 24 and _lib.Config.first_game.offset == 40
    assert _lib.lib().azg_abi_version() == 1


def test_errors_are_loud_without_device():
    # a null config must be rejected with a message, never silently ignored
    L = _lib.lib()
    h = ctypes.c_void_p()
    assert L.azg_create(None, None, ctypes.byref(h)) == -1
    assert b"null" in L.azg_last_error()


def test_small_mfma_layout_matches_python_mirror():
    """tools/small_probes.small_mfma_layout (used to pack the weights without a library call) = the
    probe library's azg_small_mfma_layout for the boards' layers (no GPU needed)."""
    import ctypes
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import small_probes as sp
    from small_probes import small_mfma_layout
    L = sp.lib()
    for H, pad, c12 in [(7, 1, 1), (7, 0, 0), (5, 0, 0), (6, 1, 1), (6, 0, 0), (4, 0, 0), (8, 1, 1), (8, 0, 0),
                        (6, 0, 1)]:
        out = (ctypes.c_int32 * 4)()
        rc = L.azg_small_mfma_layout(H, pad, 512, 512, c12, out)
        lay = small_mfma_layout(H, pad, 512, 512, bool(c12))
        if rc == 0 and tuple(out)[2] in (9, 36):
            assert lay == tuple(out)[:3], (H, pad, c12)
        else:
            assert lay is None, (H, pad, c12, rc, tuple(out))
