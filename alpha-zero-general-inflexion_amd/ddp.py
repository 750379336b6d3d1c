"""Data-parallel NNetWrapper.train over the ranks of a torch.distributed group (RCCL on ROCm).

The reference trains on one device (inflexion/pytorch/NNet.py:36-76): per epoch,
len(examples) // batch_size steps, each on a batch drawn with replacement by
`np.random.randint(len(examples), size=batch_size)` from numpy's global stream
(NNet.py:52), losses l_pi = -sum(t * log p) / B and l_v = sum((t - v)^2) / B
(NNet.py:96-100), one Adam step.  Here every rank holds the same examples and
draws the same batch indices (rank 0's numpy stream, broadcast once), takes its
own 1/N slice of each batch, and the N ranks together compute exactly the
reference step's quantities:

  * BatchNorm statistics over the whole batch, not the slice: each BatchNorm
    layer all-reduces its per-channel (sum, sum of squares) in f64 and normalises
    with the batch's mean and biased variance; the running statistics take the
    batch's unbiased variance, as nn.BatchNorm does.  The all-reduce is
    differentiable (its backward all-reduces the gradient), so the backward pass
    through the batch statistics is the whole batch's too;
  * each rank's loss is its slice's share of the batch sums divided by the global
    B, so the sum over ranks of the per-rank gradients is the batch gradient: one
    SUM all-reduce of all gradients (one flat buffer, the two loss values riding
    in its tail) per step;
  * every rank then takes the identical Adam step on the identical gradient, so the
    weights stay bitwise equal on all ranks and need no broadcast afterwards.

The arithmetic is the reference step's up to summation order (tests/test_ddp_gloo.py
compares the trained weights with the single-process trainer's within the GPU trainer's
tolerance, tests/test_gpu_train.py); at world size 1 NNetWrapper.train_examples is the
single-process trainer itself, bit-identical to the reference on the CPU
(tests/test_train_golden.py).
"""
import numpy as np
import torch
import torch.distributed as dist
import torch.nn as nn
from torch._utils import _flatten_dense_tensors, _unflatten_dense_tensors

from .dist import group_src


# collective accounting of a running train_examples_dp (its `stats` dict), else None
_STATS = None


def _count(key, nbytes):
    if _STATS is not None:
        _STATS[key + "_calls"] = _STATS.get(key + "_calls", 0) + 1
        _STATS[key + "_bytes"] = _STATS.get(key + "_bytes", 0) + int(nbytes)


class _AllReduceSum(torch.autograd.Function):
    """SUM all-reduce whose backward all-reduces the gradient (the loss is the sum of the
    ranks' losses, each of which reads the reduced value)."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        y = x.clone()
        dist.all_reduce(y, op=dist.ReduceOp.SUM, group=group)
        _count("bn_allreduce", y.numel() * y.element_size())
        return y

    @staticmethod
    def backward(ctx, g):
        g = g.clone()
        dist.all_reduce(g, op=dist.ReduceOp.SUM, group=ctx.group)
        _count("bn_allreduce", g.numel() * g.element_size())
        return g, None


class GlobalBatchNorm(nn.Module):
    """A BatchNorm1d/2d whose training-mode statistics are those of the whole data-parallel
    batch (all ranks' slices).  Shares the wrapped module's parameters and buffers; eval mode
    is the wrapped module itself."""

    def __init__(self, bn, group, world):
        super().__init__()
        self.bn = bn
        self.group = group
        self.world = world

    def forward(self, x):
        bn = self.bn
        if not bn.training:
            return bn(x)
        C = x.shape[1]
        dims = [0] + list(range(2, x.dim()))
        xd = x.double()
        stats = torch.cat([xd.sum(dims), (xd * xd).sum(dims)])
        stats = _AllReduceSum.apply(stats, self.group)
        n = (x.numel() // C) * self.world  # every rank holds an equal slice
        mean = stats[:C] / n
        var = (stats[C:] / n - mean * mean).clamp_min(0.0)
        invstd = torch.rsqrt(var + bn.eps)
        scale = (bn.weight.double() * invstd)
        shift = bn.bias.double() - mean * scale
        shape = [1, C] + [1] * (x.dim() - 2)
        y = x * scale.float().view(shape) + shift.float().view(shape)
        if bn.track_running_stats:
            with torch.no_grad():
                m = bn.momentum
                bn.running_mean.mul_(1.0 - m).add_(mean.float(), alpha=m)
                bn.running_var.mul_(1.0 - m).add_((var * (n / max(n - 1, 1))).float(), alpha=m)
                bn.num_batches_tracked.add_(1)
        return y


def _swap_batchnorms(module, group, world):
    """Replace every BatchNorm child by GlobalBatchNorm; returns the list to restore."""
    swapped = []
    for name, child in list(module.named_children()):
        if isinstance(child, nn.modules.batchnorm._BatchNorm):
            setattr(module, name, GlobalBatchNorm(child, group, world))
            swapped.append((module, name, child))
        else:
            swapped += _swap_batchnorms(child, group, world)
    return swapped


def broadcast_numpy_rng(src=0, group=None, device=None):
    """Make numpy's global RandomState on every rank equal to rank `src`'s (the batch draws
    of NNet.py:52 then agree on all ranks, and after training every rank's stream is where a
    single-process trainer would have left it)."""
    st = np.random.get_state()
    dev = device if device is not None else torch.device("cpu")
    buf = torch.zeros(626, dtype=torch.int64, device=dev)
    if dist.get_rank(group) == src:
        buf[:624] = torch.from_numpy(st[1].astype(np.int64))
        buf[624] = int(st[2])
        buf[625] = int(st[3])
    dist.broadcast(buf, src=group_src(group, src), group=group)
    b = buf.cpu().numpy()
    np.random.set_state((st[0], b[:624].astype(np.uint32), int(b[624]), int(b[625]), float(st[4])))


def broadcast_perm(perm, src=0, group=None, device=None):
    """Rank `src`'s index permutation (Coach.py:149's shuffle) on every rank, as int64."""
    dev = device if device is not None else torch.device("cpu")
    n = torch.tensor([len(perm) if dist.get_rank(group) == src else 0], dtype=torch.int64, device=dev)
    dist.broadcast(n, src=group_src(group, src), group=group)
    buf = (torch.as_tensor(perm, dtype=torch.int64, device=dev) if dist.get_rank(group) == src
           else torch.empty(int(n.item()), dtype=torch.int64, device=dev))
    dist.broadcast(buf, src=group_src(group, src), group=group)
    return buf


def broadcast_example_sets(sets, src=0, group=None, device=None):
    """Rank `src`'s list of ExampleSets (e.g. a history loadTrainExamples read on the trainer
    only) on every rank."""
    from .examples import ExampleSet
    dev = device if device is not None else torch.device("cpu")
    me = dist.get_rank(group) == src
    s = group_src(group, src)
    hdr = torch.zeros(1, dtype=torch.int64, device=dev)
    if me:
        hdr[0] = len(sets)
    dist.broadcast(hdr, src=s, group=group)
    out = []
    for i in range(int(hdr.item())):
        shp = torch.zeros(4, dtype=torch.int64, device=dev)
        if me:
            x = sets[i]
            shp.copy_(torch.tensor([len(x), x.planes.shape[1], x.planes.shape[2], x.pis.shape[1]]))
        dist.broadcast(shp, src=s, group=group)
        E, P, n, A = (int(v) for v in shp.tolist())
        if me:
            x = sets[i]
            t = [x.planes.to(dev).contiguous(), x.pis.to(dev).contiguous(), x.vs.to(dev).contiguous()]
        else:
            t = [torch.empty((E, P, n, n), device=dev), torch.empty((E, A), device=dev), torch.empty(E, device=dev)]
        for y in t:
            dist.broadcast(y, src=s, group=group)
        out.append(ExampleSet(*t))
    return out


def rank_dropout_seed(group=None, device=None):
    """A seed for this rank's dropout masks: a base drawn from rank 0's torch CPU generator,
    broadcast, plus the rank.  The reference draws an independent mask per sample of its
    batch (NNet.py:64, F.dropout in InflexionNNet.py:50-51); the ranks' slices have equal
    shapes and run the same ops, so with the generators every rank inherits (the same
    torch.manual_seed) sample i of every slice would get the same mask."""
    dev = device if device is not None else torch.device("cpu")
    buf = torch.zeros(1, dtype=torch.int64, device=dev)
    if dist.get_rank(group) == 0:
        buf[0] = int(torch.randint(0, 2**31 - 1, (1,), dtype=torch.int64).item())
    dist.broadcast(buf, src=group_src(group, 0), group=group)
    return int(buf.item()) * 1000003 + dist.get_rank(group)


def train_examples_dp(wrapper, ex, group=None, stats=None):
    """NNetWrapper.train_examples over the ranks of `group`: the reference trainer's
    epochs, batches, losses and Adam steps, each batch split evenly over the ranks
    (module docstring).  Every rank calls this with the same ExampleSet; returns the
    batches' global (l_pi, l_v) as a device tensor [batches, 2] on every rank.

    Dropout masks come from a generator state of this rank's own (rank_dropout_seed),
    forked for the duration of training: the caller's torch generators are restored.

    stats: a dict that receives the collectives' accounting (bench.py --learn-iteration):
    calls and bytes of the gradient and BatchNorm all-reduces, and the gradient
    all-reduce's time on the compute stream (HIP events on every `stats["every"]`-th step,
    default 10, milliseconds summed in grad_allreduce_ms over grad_allreduce_timed steps)."""
    dev = wrapper.device
    devices = [dev.index if dev.index is not None else torch.cuda.current_device()] if dev.type == "cuda" else []
    with torch.random.fork_rng(devices=devices):
        # drawn inside the fork: rank 0's draw does not move its restored generator
        seed = rank_dropout_seed(group, dev if dist.get_backend(group) == "nccl" else None)
        torch.default_generator.manual_seed(seed)
        if dev.type == "cuda":
            with torch.cuda.device(devices[0]):
                torch.cuda.manual_seed(seed)
        global _STATS
        _STATS = stats
        try:
            return _train_examples_dp(wrapper, ex, group, stats)
        finally:
            _STATS = None


def _train_examples_dp(wrapper, ex, group, stats=None):
    from .optim import FusedAdam
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    a = wrapper.args
    bs = int(a["batch_size"])
    if bs % world:
        raise ValueError(f"batch_size {bs} is not divisible by the {world} ranks")
    sl = bs // world
    dev = wrapper.device
    net = wrapper.nnet
    broadcast_numpy_rng(0, group, dev if dist.get_backend(group) == "nccl" else None)
    opt = wrapper._adam()
    E = len(ex)
    nb = int(E / bs)
    losses = torch.zeros((a["epochs"] * nb, 2), dtype=torch.float32, device=dev)
    planes = ex.planes.to(dev)
    pis = ex.pis.to(dev)
    vs = ex.vs.to(dev)
    params = [p for p in net.parameters() if p.requires_grad]
    swapped = _swap_batchnorms(net, group, world)
    k = 0
    try:
        for _ in range(a["epochs"]):
            net.train()
            # the epoch's batch draws in one call (the same numpy stream as nb calls) and one upload
            ids_all = np.random.randint(E, size=(nb, bs))
            mine_all = torch.from_numpy(np.ascontiguousarray(ids_all[:, rank * sl:(rank + 1) * sl])).to(dev) \
                if nb else None
            for j in range(nb):
                mine = mine_all[j]
                tp, tv = pis[mine], vs[mine]
                with wrapper._autocast():
                    out_pi, out_v = wrapper._train_forward(planes[mine])
                    l_pi = -torch.sum(tp * out_pi) / bs
                    l_v = torch.sum((tv - out_v.view(-1)) ** 2) / bs
                opt.zero_grad()
                (l_pi + l_v).backward()
                grads = [p.grad if p.grad is not None else torch.zeros_like(p) for p in params]
                flat = _flatten_dense_tensors(grads + [torch.stack([l_pi.detach(), l_v.detach()]).float()])
                timed = stats is not None and dev.type == "cuda" and k % int(stats.get("every", 10)) == 0
                if timed:
                    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    ev0.record()
                dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
                _count("grad_allreduce", flat.numel() * flat.element_size())
                if timed:
                    ev1.record()
                    stats.setdefault("_events", []).append((ev0, ev1))
                parts = _unflatten_dense_tensors(flat, grads + [losses[k]])
                if isinstance(opt, FusedAdam):
                    opt.step(grads=list(parts[:-1]))  # straight from the all-reduced buffer
                else:
                    for p, g in zip(params, parts[:-1]):
                        if p.grad is None:
                            p.grad = g.clone()
                        else:
                            p.grad.copy_(g)
                    opt.step()
                losses[k] = parts[-1]
                k += 1
    finally:
        for mod, name, child in swapped:
            setattr(mod, name, child)
    if stats is not None:
        evs = stats.pop("_events", [])
        if evs:
            torch.cuda.synchronize(dev)
            stats["grad_allreduce_ms"] = sum(a.elapsed_time(b) for a, b in evs)
            stats["grad_allreduce_timed"] = len(evs)
        stats["steps"] = k
    return losses


__all__ = ["GlobalBatchNorm", "broadcast_numpy_rng", "broadcast_perm", "broadcast_example_sets",
           "rank_dropout_seed", "train_examples_dp"]
