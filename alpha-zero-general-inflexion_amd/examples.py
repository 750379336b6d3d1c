"""Training examples on the GPU: the consumer side of the self-play hot path.

The reference builds its examples on the host while a game is played
(Coach.executeEpisode, Coach.py:74-90): per move, game.symmetries() of the
planes and of the policy plane (InflexionGame.py:102-113; 36 forms for 7x7
Inflexion, 8 for Othello), labelled with +-outcome.value at the end; learn()
keeps the last maxlenOfQueue examples of an iteration in a deque
(Coach.py:107) and trains on them (NNet.py:36-76) as f32 tensors.

Here the same list is produced by libazg's azg_examples from the compact
move records the engine (or the rank gather, dist.py) already holds: every
game is replayed from the initial position on the GPU and the kept window is
written straight into f32 device tensors in the trainer's input format --
the planes, pis and vs that NNet.train would build with
torch.FloatTensor(np.array(...)).  Nothing goes through host memory.

`ExampleSet.to_list()` converts back to the reference's list of
(board int64 ndarray, pi list, z) tuples (Coach.py:89-90), e.g. for the
`checkpoint_{i}.pth.tar.examples` pickle (Coach.py:170-176); pi values there
are the f32 values the trainer sees.

The examples file (Coach.saveTrainExamples, Coach.py:170-176).  The reference pickles the
whole history -- numItersForTrainExamplesHistory windows of up to maxlenOfQueue examples
(main.py:19,27: 20 x 200,000) -- as Python tuples every iteration: at 4096 games per
iteration 1.37e9 Python floats (~44 GB of objects, ~19 GB pickled) per save.  Here each
window is written ONCE, when it is first saved, as its own array file (`save_window`: planes
in the smallest integer type that holds them exactly, pis as CSR rows -- at most
numMCTSSims nonzeros per self-play row --, vs f32; numpy .npz, no pickle), and the examples
file is a small JSON manifest naming the history's windows in order (`write_manifest`), so a
save costs O(the new window).  `read_examples_file` loads a manifest or a reference-written
pickle; `export_reference_examples` writes the reference's pickle (a list of deques of
tuples) streamed window by window, for a reference Coach to load.
"""
import ctypes
import json
import os
import pickle
import random
import uuid
from collections import deque

import numpy as np
import torch

from . import _lib
from ._lib import check

LABEL_MODES = {"reference": 0, "per_move": 1}


def game_info(game_name, n):
    """(cells, actions, planes, symmetry forms) of a supported game."""
    kind = {"inflexion": _lib.GAME_INFLEXION, "othello": _lib.GAME_OTHELLO}[game_name]
    out = (ctypes.c_int32 * 4)()
    check(_lib.lib().azg_game_info(kind, int(n), out))
    return tuple(int(x) for x in out)


class ExampleSet:
    """A block of training examples resident on one device (f32, trainer layout)."""

    def __init__(self, planes, pis, vs):
        self.planes, self.pis, self.vs = planes, pis, vs

    def __len__(self):
        return int(self.vs.shape[0])

    @staticmethod
    def cat(sets):
        sets = [s for s in sets if len(s)]
        if not sets:
            raise ValueError("no examples")
        return ExampleSet(torch.cat([s.planes for s in sets]), torch.cat([s.pis for s in sets]),
                          torch.cat([s.vs for s in sets]))

    def index(self, idx):
        return ExampleSet(self.planes[idx], self.pis[idx], self.vs[idx])

    def to_list(self):
        """Reference example tuples (board int64 [planes, n, n], pi list, z)."""
        return list(self.iter_tuples())

    def iter_tuples(self, chunk=8192):
        """to_list()'s tuples generated `chunk` examples at a time (host memory O(chunk))."""
        for c0 in range(0, len(self), chunk):
            b = self.planes[c0:c0 + chunk].cpu().numpy().astype(np.int64)
            p = self.pis[c0:c0 + chunk].cpu().numpy().astype(np.float64)
            z = [_z_value(x) for x in self.vs[c0:c0 + chunk].cpu().numpy().tolist()]
            for i in range(len(z)):
                yield b[i], p[i].tolist(), z[i]

    @staticmethod
    def from_list(examples, device):
        """Reference example tuples -> device ExampleSet (NNet.py:54-56 conversion)."""
        boards, pis, vs = zip(*examples)
        return ExampleSet(torch.as_tensor(np.array(boards).astype(np.float64), dtype=torch.float32, device=device),
                          torch.as_tensor(np.array(pis), dtype=torch.float32, device=device),
                          torch.as_tensor(np.array(vs).astype(np.float64), dtype=torch.float32, device=device))


def _z_value(x):
    """z as the reference stores it: +-result.value, an int +-1 or a float +-1e-4 (flags.py:32-36)."""
    if abs(x) == 1.0:
        return int(x)
    if abs(x) == np.float32(1e-4):
        return 1e-4 if x > 0 else -1e-4
    return float(x)


# ---------------------------------------------------------------- examples file
FILE_FORMAT = "azg-examples"
FILE_VERSION = 1
WINDOW_DIR = "examples_windows"


def shuffle_perm(n):
    """Coach.py:149's shuffle(trainExamples) as an index permutation: the order
    random.shuffle(list(range(n))) gives, drawn on the `random` module's global stream, which
    is left where random.shuffle would leave it (libazg azg_py_shuffle, host code).  Returns
    an int64 ndarray."""
    version, internal, gauss = random.getstate()
    mt = np.array(internal[:624], dtype=np.uint32)
    pos = ctypes.c_int32(internal[624])
    perm = np.arange(n, dtype=np.int64)
    check(_lib.lib().azg_py_shuffle(perm.ctypes.data, int(n), mt.ctypes.data, ctypes.byref(pos)))
    random.setstate((version, tuple(int(x) for x in mt) + (pos.value,), gauss))
    return perm


def _planes_int_dtype(planes):
    """The smallest integer type holding every plane value exactly (planes are counts and 0/1
    masks: the turn plane reaches max_turns), or None (then kept as f32)."""
    if planes.numel() == 0:
        return torch.int8
    if not torch.equal(planes, planes.round()):
        return None
    lo, hi = (float(x) for x in torch.aminmax(planes))
    for dt, lim in ((torch.int8, 127), (torch.int16, 32767), (torch.int32, 2 ** 31 - 1)):
        if -lim - 1 <= lo and hi <= lim:
            return dt
    return None


def save_window(ex, path):
    """One history window as an array file: planes (smallest exact integer type), pis as CSR
    (row_nnz u16, cols i16/i32, vals f32: the exact f32 values), vs f32.  Written to a
    temporary name and renamed, so a reader never sees half a window."""
    dev_planes = ex.planes
    pdt = _planes_int_dtype(dev_planes)
    planes = (dev_planes.to(pdt) if pdt is not None else dev_planes).cpu().numpy()
    pis = ex.pis
    A = int(pis.shape[1]) if pis.dim() == 2 else 0
    nz = pis != 0
    row_nnz = nz.sum(dim=1).to(torch.int32)
    cols = nz.nonzero()[:, 1].to(torch.int16 if A <= 32767 else torch.int32)
    vals = pis[nz]
    arrays = dict(planes=planes, planes_shape=np.array(dev_planes.shape, dtype=np.int64),
                  pis_shape=np.array(pis.shape, dtype=np.int64),
                  row_nnz=row_nnz.cpu().numpy().astype(np.uint16 if A < 65536 else np.uint32),
                  cols=cols.cpu().numpy(), vals=vals.cpu().numpy(), vs=ex.vs.cpu().numpy())
    tmp = path + ".tmp"
    with open(tmp, "wb") as f:
        np.savez(f, **arrays)
    os.replace(tmp, path)


def load_window(path, device):
    """save_window's file -> ExampleSet on `device` (f32, the trainer's layout)."""
    with np.load(path, allow_pickle=False) as z:
        planes = torch.as_tensor(z["planes"]).to(device).float().reshape(tuple(z["planes_shape"].tolist()))
        E, A = (int(x) for x in z["pis_shape"])
        row_nnz = torch.as_tensor(z["row_nnz"].astype(np.int64)).to(device)
        cols = torch.as_tensor(z["cols"].astype(np.int64)).to(device)
        vals = torch.as_tensor(z["vals"]).to(device)
        vs = torch.as_tensor(z["vs"]).to(device)
    pis = torch.zeros((E, A), dtype=torch.float32, device=device)
    rows = torch.repeat_interleave(torch.arange(E, device=device), row_nnz)
    pis[rows, cols] = vals
    return ExampleSet(planes, pis, vs)


def write_manifest(history, filename, maxlen=None, iteration=None):
    """The examples file: a JSON manifest of the history's windows in order, each window saved
    under <folder>/examples_windows/ the first time it is written (later saves name the same
    file: O(new windows) per save).  history: ExampleSets (a loaded or saved one remembers its
    file in `saved_path`).  Returns the number of windows written by this call."""
    folder = os.path.dirname(os.path.abspath(filename))
    wdir = os.path.join(folder, WINDOW_DIR)
    os.makedirs(wdir, exist_ok=True)
    written, entries = 0, []
    for h in history:
        if not isinstance(h, ExampleSet):
            raise TypeError("write_manifest: the history holds ExampleSets (Coach.trainExamplesHistory)")
        path = getattr(h, "saved_path", None)
        if path is None or not os.path.isfile(path):
            path = os.path.join(wdir, f"w_{uuid.uuid4().hex}.npz")
            save_window(h, path)
            h.saved_path = path
            written += 1
        entries.append({"file": os.path.relpath(path, folder), "examples": len(h)})
    doc = {"format": FILE_FORMAT, "version": FILE_VERSION, "iteration": iteration, "maxlen": maxlen,
           "windows": entries}
    tmp = filename + ".tmp"
    with open(tmp, "w") as f:
        json.dump(doc, f)
    os.replace(tmp, filename)
    return written


def is_manifest(filename):
    with open(filename, "rb") as f:
        head = f.read(1)
    return head == b"{"


def read_examples_file(filename, device, maxlen=None):
    """An examples file -> list of device ExampleSets (empty windows dropped): a manifest
    (write_manifest) or the reference's pickle (Coach.py:175-176, a list of deques of
    (board, pi, z) tuples).  A reference pickle is unpickled as the reference's own
    loadTrainExamples does (Coach.py:189) -- open only files you or a reference Coach wrote."""
    if is_manifest(filename):
        with open(filename) as f:
            doc = json.load(f)
        if doc.get("format") != FILE_FORMAT or int(doc.get("version", 0)) > FILE_VERSION:
            raise ValueError(f"{filename}: not an {FILE_FORMAT} v{FILE_VERSION} manifest")
        folder = os.path.dirname(os.path.abspath(filename))
        out = []
        for w in doc["windows"]:
            path = os.path.join(folder, w["file"])
            ex = load_window(path, device)
            if len(ex) != int(w["examples"]):
                raise ValueError(f"{path}: {len(ex)} examples, the manifest says {w['examples']}")
            ex.saved_path = path
            if len(ex):
                out.append(ex)
        return out
    with open(filename, "rb") as f:
        hist = pickle.Unpickler(f).load()
    return [ExampleSet.from_list(list(h), device) for h in hist if len(h)]


class _StreamedDeque:
    """Pickles as deque(window's tuples, maxlen) -- the deque's own reduce form (type, ((),
    maxlen), None, item iterator) -- with the items generated chunk by chunk."""

    def __init__(self, ex, maxlen):
        self.ex, self.maxlen = ex, maxlen

    def __reduce_ex__(self, protocol):
        return (deque, ((), self.maxlen), None, self.ex.iter_tuples())


def export_reference_examples(history, filename, maxlen):
    """The reference's examples file (Coach.py:170-176: Pickler(f).dump(trainExamplesHistory), a
    list of deques of (board int64 ndarray, pi list, z) tuples) from device ExampleSets, for a
    reference Coach's loadTrainExamples.  Streamed: the pickler runs in fast mode (no memo, so
    written tuples are freed) over windows whose tuples are generated in chunks, so host memory
    stays O(chunk) instead of the whole history's Python objects."""
    tmp = filename + ".tmp"
    with open(tmp, "wb", buffering=1 << 24) as f:
        p = pickle.Pickler(f)
        p.fast = True
        p.dump([_StreamedDeque(h, maxlen) for h in history])
    os.replace(tmp, filename)


def examples_from_records(game_name, n, max_turns, temp_threshold, moves, actions, counts,
                          label_mode="reference", maxlen=200000):
    """ExampleSet of the finished games in the records (device tensors: moves [G]
    int32, actions [G, MM] int32, counts [G, R, A] int16 or int32 with R = MM, or R >=
    temp_threshold - 1: the temperature-1 moves' rows only, as the rank gather sends them), in game
    order, last `maxlen` kept (deque(maxlen=args.maxlenOfQueue), Coach.py:107)."""
    if label_mode not in LABEL_MODES:
        raise ValueError(f"unknown label_mode {label_mode!r}")
    cells, A, nplanes, nsym = game_info(game_name, n)
    dev = moves.device
    if dev.type != "cuda":
        raise _lib.AzgError("examples_from_records needs device tensors (no CPU fallback)")
    G, MM = actions.shape
    R = counts.shape[1] if counts.dim() == 3 else -1
    if counts.dim() != 3 or counts.shape[0] != G or counts.shape[2] != A or not (
            R == MM or min(MM, max(int(temp_threshold) - 1, 0)) <= R < MM) or moves.shape != (G,):
        raise ValueError(f"record shapes {tuple(moves.shape)} {tuple(actions.shape)} {tuple(counts.shape)} "
                         f"do not match {game_name}({n})")
    moves = moves.to(torch.int32).contiguous()
    actions = actions.to(torch.int32).contiguous()
    if counts.dtype not in (torch.int16, torch.int32):
        counts = counts.to(torch.int32)
    counts = counts.contiguous()
    upper = int(nsym * int(moves.clamp(min=0).sum().item()))
    cap = max(0, min(int(maxlen), upper))
    planes = torch.empty((cap, nplanes, n, n), dtype=torch.float32, device=dev)
    pis = torch.empty((cap, A), dtype=torch.float32, device=dev)
    vs = torch.empty((cap,), dtype=torch.float32, device=dev)
    kind = {"inflexion": _lib.GAME_INFLEXION, "othello": _lib.GAME_OTHELLO}[game_name]
    cnt = ctypes.c_int64()
    with torch.cuda.device(dev):
        stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        check(_lib.lib().azg_examples_rows(kind, int(n), int(max_turns), int(temp_threshold), G, MM,
                                           ctypes.c_void_p(moves.data_ptr()), ctypes.c_void_p(actions.data_ptr()),
                                           ctypes.c_void_p(counts.data_ptr()) if counts.numel() else None, R,
                                           counts.element_size(),
                                      LABEL_MODES[label_mode], cap, ctypes.c_void_p(planes.data_ptr()),
                                      ctypes.c_void_p(pis.data_ptr()), ctypes.c_void_p(vs.data_ptr()),
                                      ctypes.byref(cnt), stream))
    k = cnt.value
    return ExampleSet(planes[:k], pis[:k], vs[:k])


def engine_examples(engine, temp_threshold, label_mode="reference", maxlen=200000):
    """Examples of the games an engine has played (zero-copy from its records)."""
    from .dist import engine_records
    moves, actions, counts = engine_records(engine)
    if counts is None:
        raise _lib.AzgError("engine was created with record=False: no root counts to build examples from")
    max_turns = engine.cfg.max_turns
    return examples_from_records(engine.game, engine.n, max_turns, temp_threshold, moves, actions, counts,
                                 label_mode, maxlen)
