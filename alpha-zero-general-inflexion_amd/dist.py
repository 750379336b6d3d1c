"""Multi-GPU self-play: one process per GPU, games sharded by global index.

Self-play needs no communication (each game slot is independent and seeded by
its global index, so results do not depend on the GPU count).  Once per
iteration -- where the reference's Coach.learn (Coach.py:102-153) collects the
iteration's examples and trains -- the records cross ranks over RCCL (backend
"nccl" on ROCm) on xGMI:

  * with the data-parallel trainer (Coach.learn's default with several ranks,
    ddp.py): an all-gather of every rank's compact move records, so every rank
    builds the same examples; training then keeps the weights equal on every
    rank (one gradient all-reduce per step), so no weight broadcast follows;
  * with the single-rank trainer (args.distributedTrain "rank0"): a gather of
    the records to the trainer rank (an all_reduce of the sizes, then gathers
    into the trainer only) and, after training, a broadcast of the trainer's
    weights (one flat f32 buffer, ~50 MB).

A compact move record is (moves made, actions, root visit counts) per game:
enough to rebuild every training example (Coach.py:74-90) by replaying the
actions from the initial position (examples.examples_from_records; temperatures
follow from tempThreshold).  The counts travel sparse: only the moves played at
temperature 1 need them (a temperature-0 move's pi is the one-hot of its action,
MCTS.py:51-56), and of a root's 343 counts only the visited actions are nonzero
(at most sims + the subtree kept from the previous move), so each such move is
sent as its number of visited actions plus (action, count) pairs packed in 32
bits.  At 4096 games x 344 moves (tempThreshold 30: 29 moves with counts, ~10
visited actions each) that is ~5 MB of counts, ~8 MB with the int16 actions, per
rank instead of 0.97 GB of dense int16 counts.
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


def gather_records(engine, dst=0, group=None, temp_threshold=None):
    """Gather compact move records of all ranks (moves made so far) to `dst`.
    Returns (moves [W*G], actions [W*G, m], counts [W*G, m, A] int16/int32) on dst, None
    elsewhere (dst=None: on every rank), and the bytes this rank sent.  temp_threshold:
    see gather_record_tensors (default: the engine's own) -- the counts of moves at or
    past tempThreshold - 1 come back as zeros."""
    moves, actions, counts = engine_records(engine)
    tt = engine.cfg.temp_threshold if temp_threshold is None else temp_threshold
    return gather_record_tensors(moves, actions, counts, dst, group, actions_per_move=engine.A, temp_threshold=tt)


def group_src(group, rank):
    """Global rank of `rank` in `group` (torch's src/dst arguments are global ranks)."""
    if group is None or group is dist.group.WORLD:
        return int(rank)
    return dist.get_global_rank(group, int(rank))


def _gather(t, dst, group):
    """dist.gather of equal-shaped tensors into one [ws, ...] tensor on dst only
    (dst None: dist.all_gather, every rank receives)."""
    ws = dist.get_world_size(group)
    if dst is None:
        out = torch.empty((ws,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        dist.all_gather(list(out.unbind(0)), t.contiguous(), group=group)
        return out
    if dist.get_rank(group) == dst:
        out = torch.empty((ws,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        dist.gather(t, list(out.unbind(0)), dst=group_src(group, dst), group=group)
        return out
    dist.gather(t, None, dst=group_src(group, dst), group=group)
    return None


def _pad_to(t, n):
    if t.shape[0] == n:
        return t.contiguous()
    out = t.new_zeros((n,) + tuple(t.shape[1:]))
    out[:t.shape[0]] = t
    return out


def sparse_counts(moves, counts, rows):
    """Encode the first `rows` moves of every game's root counts (rows past a game's
    end are empty): (per-(game, move) number of visited actions int16 [G*rows],
    pairs [nnz] int32 = action | count << 16, or [nnz, 2] int32 when a count exceeds
    65535), in (game, move, action) order."""
    G, _, A = counts.shape
    sub = counts[:, :rows]
    live = torch.arange(rows, device=counts.device)[None, :] < moves.to(torch.int64)[:, None]
    sub = sub * live[:, :, None].to(sub.dtype)
    nz = sub != 0
    row_nnz = nz.sum(dim=2, dtype=torch.int32).reshape(-1).to(torch.int16)
    act = nz.reshape(-1, A).nonzero()[:, 1].to(torch.int32)
    val = sub[nz].to(torch.int32)
    if val.numel() and int(val.max()) > 65535:
        return row_nnz, torch.stack([act, val], dim=1)
    return row_nnz, act | (val << 16)


def dense_counts(row_nnz, pairs, G, rows, m, A, dtype):
    """Inverse of sparse_counts: [G, m, A] counts, zero outside the encoded rows."""
    out = torch.zeros((G, m, A), dtype=dtype, device=row_nnz.device)
    n = row_nnz.to(torch.int64)
    if pairs.shape[0]:
        row = torch.repeat_interleave(torch.arange(G * rows, device=n.device), n)
        if pairs.dim() == 2:
            act, val = pairs[:, 0].to(torch.int64), pairs[:, 1]
        else:
            act, val = (pairs & 0xFFFF).to(torch.int64), (pairs >> 16) & 0xFFFF
        out.view(G, m * A)[row // rows, (row % rows) * A + act] = val.to(dtype)
    return out


def gather_record_tensors(moves, actions, counts, dst=0, group=None, actions_per_move=343, temp_threshold=None):
    """gather_records on plain tensors (any device the group's backend serves).
    Only `dst` allocates and receives the other ranks' records; dst=None gives every
    rank all records (all_gather: the data-parallel trainer, where every rank builds
    the iteration's examples itself).

    temp_threshold: the counts of a move are needed only if it was played at
    temperature 1 (episodeStep < tempThreshold, Coach.py:68), so only the first
    tempThreshold - 1 moves' counts are sent; the others arrive as zeros (their
    examples' pi is the one-hot of the action).  None sends every move's counts.
    Returns ((moves [W*G], actions [W*G, m] int32, counts [W*G, rows, A] int16, or
    int32 if a count exceeds 32767) on dst, None elsewhere; the bytes this rank sent).
    rows = m without temp_threshold; with it the counts are TRUNCATED to the temperature-1
    moves, rows = min(m, tempThreshold - 1) (at 8 ranks x 4096 games
    a dense [W*G, 344, 343] int16 buffer is 7.7 GB, the 29 rows that carry counts 0.65 GB) --
    exactly what examples_from_records needs, but not the full records (statistics or saving
    records need temp_threshold=None)."""
    A = counts.shape[2] if counts is not None else int(actions_per_move)
    G = moves.shape[0]
    dev = moves.device
    m_loc = int(torch.max(moves)) if G else 0
    rows_loc = m_loc if temp_threshold is None else min(m_loc, max(int(temp_threshold) - 1, 0))
    if counts is not None:
        row_nnz, pairs = sparse_counts(moves, counts[:, :m_loc], rows_loc)
    else:
        row_nnz = torch.zeros(G * rows_loc, dtype=torch.int16, device=dev)
        pairs = torch.zeros(0, dtype=torch.int32, device=dev)
    cmax = int(((pairs >> 16) & 0xFFFF).max()) if pairs.dim() == 1 and pairs.numel() else (
        int(pairs[:, 1].max()) if pairs.numel() else 0)
    hdr = torch.tensor([m_loc, cmax, pairs.shape[0], int(pairs.dim() == 2)], dtype=torch.int64, device=dev)
    hmax = hdr.clone()
    dist.all_reduce(hmax, op=dist.ReduceOp.MAX, group=group)
    m, cmax, nnz_max, wide = (int(x) for x in hmax.tolist())
    rows = m if temp_threshold is None else min(m, max(int(temp_threshold) - 1, 0))
    if wide and pairs.dim() == 1:
        pairs = torch.stack([pairs & 0xFFFF, (pairs >> 16) & 0xFFFF], dim=1)
    # every rank pads to the group's max moves / rows / pairs so the gathers are equal-shaped
    act = actions[:, :m]
    if act.shape[1] < m:
        act = torch.cat([act, act.new_zeros((G, m - act.shape[1]))], dim=1)
    act16 = act.to(torch.int16).contiguous() if A <= 32767 else act.contiguous()
    rn = row_nnz.reshape(G, rows_loc)
    rn = torch.cat([rn, rn.new_zeros((G, rows - rows_loc))], dim=1).reshape(-1) if rows > rows_loc else row_nnz
    pairs_p = _pad_to(pairs, nnz_max)
    mv = moves.to(torch.int32).contiguous()
    out_hdr = _gather(hdr, dst, group)
    out_mv = _gather(mv, dst, group)
    out_act = _gather(act16.view(torch.uint8), dst, group)  # raw bytes: RCCL/gloo have no int16
    out_rn = _gather(rn.contiguous().view(torch.uint8), dst, group)
    out_pairs = _gather(pairs_p.view(torch.uint8), dst, group)
    sent = (hdr.numel() * 8 + mv.numel() * 4 + act16.numel() * act16.element_size() + rn.numel() * 2
            + pairs_p.numel() * 4)
    if out_mv is None:
        return None, sent
    W = out_mv.shape[0]
    ctype = torch.int16 if cmax <= 32767 else torch.int32
    acts = out_act.view(act16.dtype).reshape(W * G, m).to(torch.int32)
    cnts = torch.empty((W * G, rows, A), dtype=ctype, device=out_mv.device)
    ptype_rows = 2 if wide else 1
    for r in range(W):
        nnz_r = int(out_hdr[r, 2])
        pr = out_pairs[r].view(torch.int32).reshape(nnz_max, ptype_rows) if wide else out_pairs[r].view(torch.int32)
        cnts[r * G:(r + 1) * G] = dense_counts(out_rn[r].view(torch.int16), pr[:nnz_r], G, rows, rows, A, ctype)
    return (out_mv.reshape(-1), acts, cnts), sent


def dense_record_bytes(G, m, A):
    """Bytes the round-2 gather sent per rank: moves i32, actions i32, dense int16 counts."""
    return G * 4 + G * m * 4 + G * m * A * 2


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
    with torch.no_grad():  # in-place copies that bump the tensors' version counters (mcts.fast_evaluator)
        for t, f in zip(f32, _unflatten_dense_tensors(flat, [t.data for t in f32])):
            t.copy_(f)
    nbytes = flat.numel() * 4
    if rest:
        ints = torch.cat([t.data.reshape(-1).to(torch.int64) for t in rest])
        dist.broadcast(ints, src=src, group=group)
        off = 0
        with torch.no_grad():
            for t in rest:
                t.copy_(ints[off:off + t.numel()].reshape(t.shape).to(t.dtype))
                off += t.numel()
        nbytes += ints.numel() * 8
    return nbytes


def iteration_sync(engine, module, trainer=0, group=None, mode="ddp"):
    """The per-iteration exchange of configs[3] as Coach.learn runs it: "ddp" (the default
    with several ranks) all-gathers the records to every rank; "rank0" gathers them to the
    trainer and broadcasts its weights.  Returns the bytes this rank sent."""
    if mode == "ddp":
        return gather_records(engine, dst=None, group=group)[1]
    if mode != "rank0":
        raise ValueError(f"unknown iteration_sync mode {mode!r}")
    _, sent = gather_records(engine, dst=trainer, group=group)
    wb = broadcast_weights(module, src=trainer, group=group)
    return sent + wb
