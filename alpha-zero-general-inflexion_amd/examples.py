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
"""
import ctypes

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
        b = self.planes.cpu().numpy().astype(np.int64)
        p = self.pis.cpu().numpy().astype(np.float64)
        v = self.vs.cpu().numpy()
        # z is +-result.value: int +-1 or float +-1e-4 (flags.py:32-36), restored exactly
        z = [int(x) if abs(x) == 1.0 else (1e-4 if x > 0 else -1e-4) if abs(x) == np.float32(1e-4) else float(x)
             for x in v.tolist()]
        return [(b[i], p[i].tolist(), z[i]) for i in range(len(z))]

    @staticmethod
    def from_list(examples, device):
        """Reference example tuples -> device ExampleSet (NNet.py:54-56 conversion)."""
        boards, pis, vs = zip(*examples)
        return ExampleSet(torch.as_tensor(np.array(boards).astype(np.float64), dtype=torch.float32, device=device),
                          torch.as_tensor(np.array(pis), dtype=torch.float32, device=device),
                          torch.as_tensor(np.array(vs).astype(np.float64), dtype=torch.float32, device=device))


def examples_from_records(game_name, n, max_turns, temp_threshold, moves, actions, counts,
                          label_mode="reference", maxlen=200000):
    """ExampleSet of the finished games in the records (device tensors: moves [G]
    int32, actions [G, MM] int32, counts [G, MM, A] int16 or int32), in game order,
    last `maxlen` kept (deque(maxlen=args.maxlenOfQueue), Coach.py:107)."""
    if label_mode not in LABEL_MODES:
        raise ValueError(f"unknown label_mode {label_mode!r}")
    cells, A, nplanes, nsym = game_info(game_name, n)
    dev = moves.device
    if dev.type != "cuda":
        raise _lib.AzgError("examples_from_records needs device tensors (no CPU fallback)")
    G, MM = actions.shape
    if counts.shape != (G, MM, A) or moves.shape != (G,):
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
        check(_lib.lib().azg_examples(kind, int(n), int(max_turns), int(temp_threshold), G, MM,
                                      ctypes.c_void_p(moves.data_ptr()), ctypes.c_void_p(actions.data_ptr()),
                                      ctypes.c_void_p(counts.data_ptr()), counts.element_size(),
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
