"""Multi-GPU self-play: one process per GPU, games sharded by global index.

Self-play needs no communication (each game slot is independent and seeded by
its global index, so results do not depend on the GPU count).  Once per
iteration -- where the reference's Coach.learn (Coach.py:102-153) collects the
iteration's examples and trains -- two collectives run over RCCL (backend
"nccl" on ROCm) on xGMI:

  * gather of every rank's compact move records to the trainer rank
    (an all_reduce of the sizes, then gathers into the trainer only);
  * broadcast of the trainer's weights (one flat f32 buffer, ~50 MB).

A compact move record is (moves made, actions, root visit counts as int16 --
int32 if any count exceeds 32767) per game: enough to rebuild every training
example (Coach.py:74-90) by replaying the actions from the initial position
(examples.examples_from_records; temperatures follow from tempThreshold).
"""
import ctypes

import torch
import torch.distributed as dist
from torch._utils import _flatten_dense_tensors, _unflatten_dense_tensors

from . import _lib


class _DevArray:
    """Zero-copy view of an engine-owned device buffer as a torch tensor."""

    def __init__(self, ptr, shape, typestr):
        self.__cuda_array_interface__ = {"shape": tuple(shape), "typestr": typestr, "data": (int(ptr), False),
                                         "version": 3, "strides": None}


def engine_records(engine):
    """(moves [G] i32, actions [G,MM] i32, counts [G,MM,A] i32 or None) as device tensors (no copy)."""
    ptrs = (ctypes.c_void_p * 8)()
    _lib.check(engine.L.azg_device_ptrs(engine.h, ptrs))
    dev = engine.device
    G, MM = engine.G, engine.max_moves
    moves = torch.as_tensor(_DevArray(ptrs[7], (G,), "<i4"), device=dev)
    actions = torch.as_tensor(_DevArray(ptrs[5], (G, MM), "<i4"), device=dev)
    counts = None
    if ptrs[6]:
        counts = torch.as_tensor(_DevArray(ptrs[6], (G, MM, engine.A), "<i4"), device=dev)
    return moves, actions, counts


def gather_records(engine, dst=0, group=None):
    """Gather compact move records of all ranks (moves made so far) to `dst`.
    Returns (moves [W*G], actions [W*G, m], counts [W*G, m, A] int16/int32) on dst, None
    elsewhere, and the bytes this rank sent."""
    moves, actions, counts = engine_records(engine)
    return gather_record_tensors(moves, actions, counts, dst, group, actions_per_move=engine.A)


def group_src(group, rank):
    """Global rank of `rank` in `group` (torch's src/dst arguments are global ranks)."""
    if group is None or group is dist.group.WORLD:
        return int(rank)
    return dist.get_global_rank(group, int(rank))


def _gather(t, dst, group):
    """dist.gather of equal-shaped tensors into one [ws, ...] tensor on dst only."""
    ws = dist.get_world_size(group)
    if dist.get_rank(group) == dst:
        out = torch.empty((ws,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        dist.gather(t, list(out.unbind(0)), dst=group_src(group, dst), group=group)
        return out
    dist.gather(t, None, dst=group_src(group, dst), group=group)
    return None


def gather_record_tensors(moves, actions, counts, dst=0, group=None, actions_per_move=343):
    """gather_records on plain tensors (any device the group's backend serves).
    Only `dst` allocates and receives the other ranks' records."""
    A = counts.shape[2] if counts is not None else int(actions_per_move)
    m_local = torch.stack([torch.max(moves).to(torch.int64),
                           (counts.max() if counts is not None and counts.numel() else moves.new_zeros(())).to(
                               torch.int64)])
    m_all = m_local.clone()
    dist.all_reduce(m_all, op=dist.ReduceOp.MAX, group=group)
    m, cmax = (int(x) for x in m_all.tolist())
    ctype = torch.int16 if cmax <= 32767 else torch.int32
    G = moves.shape[0]
    act = actions[:, :m].contiguous()
    cnt = counts[:, :m].to(ctype).contiguous() if counts is not None else torch.zeros(
        (G, m, A), dtype=ctype, device=moves.device)
    mv = moves.contiguous()
    out_mv = _gather(mv, dst, group)
    out_act = _gather(act, dst, group)
    # moved as raw bytes (RCCL/gloo have no int16 type)
    out_cnt = _gather(cnt.view(torch.uint8), dst, group)
    sent = mv.numel() * 4 + act.numel() * 4 + cnt.numel() * cnt.element_size()
    if out_mv is not None:
        return (out_mv.reshape(-1), out_act.reshape(-1, m), out_cnt.view(ctype).reshape(-1, m, A)), sent
    return None, sent


def broadcast_weights(module, src=0, group=None):
    """Broadcast every parameter and buffer of `module` from `src` (a rank of `group`):
    the f32 ones as one flat buffer, the rest (BatchNorm's num_batches_tracked) as one
    int64 buffer."""
    src = group_src(group, src)
    tensors = list(module.parameters()) + list(module.buffers())
    f32 = [t for t in tensors if t.dtype == torch.float32]
    rest = [t for t in tensors if t.dtype != torch.float32]
    flat = _flatten_dense_tensors([t.data for t in f32])
    dist.broadcast(flat, src=src, group=group)
    for t, f in zip(f32, _unflatten_dense_tensors(flat, [t.data for t in f32])):
        t.data.copy_(f)
    nbytes = flat.numel() * 4
    if rest:
        ints = torch.cat([t.data.reshape(-1).to(torch.int64) for t in rest])
        dist.broadcast(ints, src=src, group=group)
        off = 0
        for t in rest:
            t.data.copy_(ints[off:off + t.numel()].reshape(t.shape).to(t.dtype))
            off += t.numel()
        nbytes += ints.numel() * 8
    return nbytes


def iteration_sync(engine, module, trainer=0, group=None):
    """The per-iteration exchange of configs[3]: examples in, weights out."""
    _, sent = gather_records(engine, dst=trainer, group=group)
    wb = broadcast_weights(module, src=trainer, group=group)
    return sent + wb
