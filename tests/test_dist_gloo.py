"""Multi-process (world size 2, gloo, CPU) tests of the per-iteration exchange:
move-record gather to the trainer rank and weight broadcast from it."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import azg_amd  # noqa: F401
        from azg_amd import dist as ad
        from azg_amd.nnet import InflexionNNet
        G, MM = 3, 10
        moves = torch.tensor([4 + rank, 2, 6 - rank], dtype=torch.int32)
        actions = torch.arange(G * MM, dtype=torch.int32).reshape(G, MM) + 1000 * rank
        counts = (torch.arange(G * MM * 343, dtype=torch.int32).reshape(G, MM, 343) % 97) + rank
        out, sent = ad.gather_record_tensors(moves, actions, counts, dst=0)
        res = {"sent": sent, "none_off_dst": out is None}
        if rank == 0:
            mv, act, cnt = out
            res["moves"] = mv.tolist()
            res["m"] = act.shape[1]
            res["act_ok"] = all(torch.equal(act[r * G:(r + 1) * G], (torch.arange(G * MM).reshape(G, MM)
                                 + 1000 * r)[:, :act.shape[1]].int()) for r in range(world))
            # rank 1's counts, zero past each game's end (moves [5, 2, 5])
            live = torch.arange(act.shape[1])[None, :, None] < torch.tensor([5, 2, 5])[:, None, None]
            res["cnt_ok"] = torch.equal(cnt[G:2 * G].long(), torch.where(
                live, (torch.arange(G * MM * 343).reshape(G, MM, 343) % 97 + 1)[:, :act.shape[1]], 0))
        torch.manual_seed(rank)  # different weights per rank before the broadcast
        net = InflexionNNet(num_channels=16)
        nbytes = ad.broadcast_weights(net, src=0)
        torch.manual_seed(0)
        ref = InflexionNNet(num_channels=16)
        res["bcast_ok"] = all(torch.equal(a, b) for a, b in zip(net.state_dict().values(),
                                                                  ref.state_dict().values()))
        res["bcast_bytes"] = nbytes
        # a root count above int16: the gather switches to int32 on every rank
        big = counts.clone()
        big[0, 0, 0] = 40000 if rank == 1 else 7
        out2, sent2 = ad.gather_record_tensors(moves, actions, big, dst=0)
        res["sent2"] = sent2
        if rank == 0:
            res["big_ok"] = out2[2].dtype == torch.int32 and int(out2[2][G, 0, 0]) == 40000
        # above 16 bits: (action, count) pairs widen to 2 x 32 bits on every rank
        big[1, 1, 5] = 70000 if rank == 0 else 1
        out3, sent3 = ad.gather_record_tensors(moves, actions, big, dst=0)
        res["sent3"] = sent3
        if rank == 0:
            want = torch.cat([torch.where(torch.arange(MM)[None, :, None] < moves[:, None, None].long(), big, 0)
                              for _ in range(1)])[:, :out3[1].shape[1]]
            res["wide_ok"] = (out3[2].dtype == torch.int32 and int(out3[2][1, 1, 5]) == 70000
                              and torch.equal(out3[2][:G].long(), want.long()))
        # the trainer's skipFirstSelfPlay decides for every rank (a rank-0-only
        # loadTrainExamples must not leave the ranks in different collectives)
        from azg_amd.coach import Coach
        c = Coach(None, "stub", None)
        c.skipFirstSelfPlay = rank == 0
        res["skip"] = c.agree_skip_first()
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def _worker3(rank, world, port, q):
    """world 3, subgroup of global ranks [1, 2]: group rank 0 is global rank 1."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import azg_amd  # noqa: F401
        from azg_amd import dist as ad
        from azg_amd.coach import Coach
        from azg_amd.nnet import InflexionNNet
        grp = dist.new_group([1, 2])
        res = {}
        if rank in (1, 2):
            torch.manual_seed(rank)
            net = InflexionNNet(num_channels=8)
            ad.broadcast_weights(net, src=0, group=grp)  # group rank 0 = global rank 1
            torch.manual_seed(1)
            ref = InflexionNNet(num_channels=8)
            res["bcast_ok"] = all(torch.equal(a, b) for a, b in zip(net.state_dict().values(),
                                                                      ref.state_dict().values()))
            moves = torch.tensor([rank, rank + 1], dtype=torch.int32)
            actions = torch.full((2, 4), rank, dtype=torch.int32)
            counts = torch.full((2, 4, 5), rank, dtype=torch.int32)
            out, _ = ad.gather_record_tensors(moves, actions, counts, dst=0, group=grp)
            res["gather"] = None if out is None else out[0].tolist()
            c = Coach(None, "stub", None)
            c.skipFirstSelfPlay = rank == 1
            res["skip"] = c.agree_skip_first(grp)
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_subgroup_ranks_world3():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker3, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[1]["bcast_ok"] and res[2]["bcast_ok"]
    assert res[1]["gather"] == [1, 2, 2, 3] and res[2]["gather"] is None
    assert res[1]["skip"] is True and res[2]["skip"] is True


def test_gather_and_broadcast_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    r0 = res[0]
    assert r0["moves"] == [4, 2, 6, 5, 2, 5]
    assert r0["m"] == 6  # max moves over ranks
    assert r0["act_ok"] and r0["cnt_ok"]
    assert res[0]["bcast_ok"] and res[1]["bcast_ok"]
    assert res[1]["bcast_bytes"] == res[0]["bcast_bytes"] > 0
    assert r0["big_ok"] and r0["wide_ok"] and res[1]["sent3"] > res[1]["sent2"] == res[1]["sent"]
    assert res[1]["none_off_dst"] and not res[0]["none_off_dst"]
    assert res[0]["skip"] is True and res[1]["skip"] is True


def _worker_sparse(rank, world, port, q):
    """Realistic records (oracle self-play, the reference's search): each rank plays 3
    games; the gather sends only the temperature-1 moves' visited (action, count)
    pairs, and the trainer rebuilds exactly the examples of the original records."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import numpy as np
        import azg_amd  # noqa: F401
        import oracle_lib as ol
        from azg_amd import dist as ad
        from azg_amd.coach import examples_from_record
        from azg_amd.inflexion import InflexionGame
        G, MT, TT, A = 3, 60, 30, 343
        eps = [ol.episode(7, MT, 25, 1, TT, 50 + rank * G + i) for i in range(G)]
        MM = MT + 1
        moves = torch.tensor([e["moves"] for e in eps], dtype=torch.int32)
        actions = torch.zeros((G, MM), dtype=torch.int32)
        counts = torch.zeros((G, MM, A), dtype=torch.int32)
        for i, e in enumerate(eps):
            actions[i, :e["moves"]] = torch.from_numpy(e["actions"])
            counts[i, :e["moves"]] = torch.from_numpy(e["counts"])
        out, sent = ad.gather_record_tensors(moves, actions, counts, dst=0, temp_threshold=TT)
        res = {"sent": sent, "dense": ad.dense_record_bytes(G, int(moves.max()), A)}
        if rank == 0:
            mv, act, cnt = out
            res["count_rows"], res["max_moves"] = int(cnt.shape[1]), int(act.shape[1])
            game = InflexionGame(7, max_turns=MT, max_power=6)
            same = True
            for r in range(world):
                for i in range(G):
                    e = ol.episode(7, MT, 25, 1, TT, 50 + r * G + i)
                    m = e["moves"]
                    k = r * G + i
                    temps = (np.arange(m) + 1 < TT).astype(np.int8)
                    a = examples_from_record(game, e["actions"], temps, e["counts"], m)
                    b = examples_from_record(game, act[k].numpy(), temps, cnt[k].numpy(), int(mv[k]))
                    same &= len(a) == len(b) and all(
                        np.array_equal(x[0], y[0]) and x[1] == y[1] and x[2] == y[2] for x, y in zip(a, b))
                    nt = min(m, TT - 1)
                    same &= np.array_equal(cnt[k, :nt].numpy(), e["counts"][:nt])
            res["same"] = bool(same)
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_sparse_gather_rebuilds_examples_world2(world):
    """(world 8, VERDICT r05: the 8-GPU node's rank count) every rank's games gathered to rank 0
    equal the records of one process holding all 8 x 3 games, move for move."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_sparse, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0]["same"]
    assert res[0]["count_rows"] == min(res[0]["max_moves"], 29)  # only the temperature-1 rows are allocated
    for r in range(world):  # <= 15% of the dense int16 gather
        assert res[r]["sent"] <= 0.15 * res[r]["dense"], (res[r]["sent"], res[r]["dense"])


def _host_fail_worker(rank, world, port, q):
    """Rank 1's host self-play raises; every rank must raise instead of rank 0 waiting in the gather."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import azg_amd  # noqa: F401
        from azg_amd.coach import Coach

        class A(dict):
            __getattr__ = dict.__getitem__
        c = Coach(None, "stub", A(numEps=1, maxlenOfQueue=100, numMCTSSims=2, cpuct=1, tempThreshold=1))

        def host(num_games, seed_base, first_game, evaluator=None):
            if rank == 1:
                raise ValueError("rank 1 failed")
            return []
        c._host_selfplay = host
        try:
            c._host_selfplay_iteration(0, 1, None, True)
            q.put((rank, "returned"))
        except ValueError as e:
            q.put((rank, f"ValueError {e}"))
        except RuntimeError as e:
            q.put((rank, f"RuntimeError {e}"))
    finally:
        dist.destroy_process_group()


def test_host_selfplay_failure_reaches_every_rank():
    """the multi-rank host path (plugins without native rules) agrees on failure
    before its object gather, as the native path does: the failing rank re-raises its error,
    the others raise too instead of blocking until the process group's timeout."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_host_fail_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res[1] == "ValueError rank 1 failed"
    assert res[0].startswith("RuntimeError host self-play failed on another rank")
