"""Probe: C4's 4096 games as two half-batch engines on two HIP streams, the persistent
split GEMM capped at fewer CUs (azg_set_gemm_blocks), so that one half's GEMM (MFMA-bound)
can run beside the other half's Winograd transforms (HBM-bound).  Prints one JSON line
per arrangement, alternating rounds in one process (rule: interleaved A/B)."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import azg_amd  # noqa: E402,F401
from azg_amd import _lib  # noqa: E402
from azg_amd.engine import SelfPlayEngine  # noqa: E402
from azg_amd.nnet import InferenceNet, InflexionNNet  # noqa: E402


def run_one(eng, moves):
    torch.cuda.synchronize()
    e0 = eng.stats()["expansions"]
    t0 = time.perf_counter()
    for _ in range(moves):
        eng.move()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return (eng.stats()["expansions"] - e0) / dt, dt / moves * 1e3


def run_two(engs, streams, moves):
    torch.cuda.synchronize()
    e0 = sum(e.stats()["expansions"] for e in engs)
    t0 = time.perf_counter()
    for _ in range(moves):
        for _ in range(engs[0].sims):
            for e, s in zip(engs, streams):
                with torch.cuda.stream(s):
                    e.simulate()
        for e, s in zip(engs, streams):
            with torch.cuda.stream(s):
                e.move_end()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return (sum(e.stats()["expansions"] for e in engs) - e0) / dt, dt / moves * 1e3


class TwoStreamNet(torch.nn.Module):
    """One engine's leaf batch as two halves, each through its own InferenceNet on its
    own stream (fork / join with events); outputs concatenated on the caller's stream."""

    def __init__(self, net, parts=2):
        super().__init__()
        self.subs = torch.nn.ModuleList([InferenceNet(net) for _ in range(parts)])
        self.streams = [torch.cuda.Stream() for _ in range(parts)]
        self.outputs_probs = True

    def forward(self, x):
        main = torch.cuda.current_stream()
        B = x.shape[0]
        n = len(self.subs)
        cuts = [B * i // n for i in range(n + 1)]
        ev = torch.cuda.Event()
        ev.record(main)
        outs = []
        for i, (sub, s) in enumerate(zip(self.subs, self.streams)):
            s.wait_event(ev)
            with torch.cuda.stream(s):
                p, v = sub(x[cuts[i]:cuts[i + 1]])
            p.record_stream(main)
            v.record_stream(main)
            outs.append((p, v))
        for s in self.streams:
            main.wait_stream(s)
        x.record_stream(self.streams[0])
        x.record_stream(self.streams[1])
        return torch.cat([p for p, _ in outs]), torch.cat([v for _, v in outs])

    def check_range(self):
        for sub in self.subs:
            sub.check_range()


def _st(e):
    torch.cuda.synchronize()
    s = e.stats()
    return {"expansions": s["expansions"], "error": s["error"], "max_live": s["max_live_nodes"]}


def diag(a):
    """Which arrangement breaks: one half-engine on a side stream, two on one stream, two
    on two streams (stub evaluator, then the network)."""
    torch.manual_seed(0)
    net = InflexionNNet().cuda().eval()
    H = a.games // 2
    for evname in ("stub", "net"):
        def mk(k, s=None):
            ev = "stub" if evname == "stub" else InferenceNet(net)
            if s is None:
                return SelfPlayEngine(H, sims=25, evaluator=ev, max_turns=343, first_game=k * H)
            with torch.cuda.stream(s):
                return SelfPlayEngine(H, sims=25, evaluator=ev, max_turns=343, first_game=k * H)
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
        e = mk(0, s1)
        with torch.cuda.stream(s1):
            e.move()
        print(json.dumps({"ev": evname, "case": "one side stream", **_st(e)}), flush=True)
        es = [mk(0), mk(1)]
        for _ in range(25):
            for x in es:
                x.simulate()
        for x in es:
            x.move_end()
        print(json.dumps({"ev": evname, "case": "two on one stream", "r": [_st(x) for x in es]}), flush=True)
        ss = [s1, s2]
        es = [mk(0, s1), mk(1, s2)]
        run_two(es, ss, 1)
        print(json.dumps({"ev": evname, "case": "two streams", "r": [_st(x) for x in es]}), flush=True)


def split_net(a):
    """One engine; its evaluator InferenceNet vs TwoStreamNet (2 and 4 parts): outputs
    bit-equal on a real leaf batch, then alternating timed rounds."""
    torch.manual_seed(0)
    net = InflexionNNet().cuda().eval()
    forms = {"inference": InferenceNet(net), "two_stream": TwoStreamNet(net, 2), "four_stream": TwoStreamNet(net, 4)}
    engs = {k: SelfPlayEngine(a.games, sims=25, evaluator=ev, max_turns=343) for k, ev in forms.items()}
    for e in engs.values():
        e.move()
    x = engs["inference"].planes.clone()
    with torch.no_grad():
        ref = forms["inference"](x)
        for k in ("two_stream", "four_stream"):
            got = forms[k](x)
            torch.cuda.synchronize()
            print(json.dumps({"form": k, "P_equal": bool(torch.equal(got[0], ref[0])),
                              "v_equal": bool(torch.equal(got[1].reshape(-1), ref[1].reshape(-1)))}), flush=True)
    res = {}
    for r in range(a.rounds):
        for k, e in engs.items():
            v, ms = run_one(e, a.moves)
            res.setdefault(k, []).append((v, ms))
        print(json.dumps({"round": r, **{k: round(x[-1][0]) for k, x in res.items()}}), flush=True)
    for k, e in engs.items():
        assert e.stats()["error"] == 0
        e.check_evaluator()
    a0 = engs["inference"].read_moves()
    for k in ("two_stream", "four_stream"):
        b0 = engs[k].read_moves()
        print(json.dumps({"form": k, "records_equal": bool((a0["counts"] == b0["counts"]).all()
                                                           and (a0["actions"] == b0["actions"]).all())}), flush=True)
    for k, x in res.items():
        vs = sorted(v for v, _ in x)
        print(json.dumps({"arrangement": k, "median_exp_per_s": vs[len(vs) // 2], "min": vs[0], "max": vs[-1],
                          "ms_per_move": sorted(m for _, m in x)[len(x) // 2]}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--games", type=int, default=4096)
    ap.add_argument("--moves", type=int, default=3)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--caps", default="0,128,160,192")
    ap.add_argument("--diag", action="store_true")
    ap.add_argument("--split-net", action="store_true")
    a = ap.parse_args()
    if a.diag:
        return diag(a)
    if a.split_net:
        return split_net(a)
    L = _lib.lib()
    torch.manual_seed(0)
    net = InflexionNNet().cuda().eval()
    G, H = a.games, a.games // 2
    one = SelfPlayEngine(G, sims=25, evaluator=InferenceNet(net), max_turns=343)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    two = []
    for k, s in enumerate(streams):
        with torch.cuda.stream(s):
            two.append(SelfPlayEngine(H, sims=25, evaluator=InferenceNet(net), max_turns=343, first_game=k * H))
    # warm up every arrangement (libraries, workspaces)
    one.move()
    torch.cuda.synchronize()
    print(json.dumps({"created": [dict(e.stats(), active=e.active()) for e in two]}), flush=True)
    for cap in [int(c) for c in a.caps.split(",")]:
        _lib.check(L.azg_set_gemm_blocks(cap))
        run_two(two, streams, 1)
        print(json.dumps({"warm": cap, "stats": [dict(e.stats(), active=e.active()) for e in two]}), flush=True)
    _lib.check(L.azg_set_gemm_blocks(0))
    res = {}
    for r in range(a.rounds):
        _lib.check(L.azg_set_gemm_blocks(0))
        v, ms = run_one(one, a.moves)
        res.setdefault("one", []).append((v, ms))
        for cap in [int(c) for c in a.caps.split(",")]:
            _lib.check(L.azg_set_gemm_blocks(cap))
            v, ms = run_two(two, streams, a.moves)
            res.setdefault(f"two_cap{cap}", []).append((v, ms))
        print(json.dumps({"round": r, **{k: round(x[-1][0]) for k, x in res.items()}}), flush=True)
    _lib.check(L.azg_set_gemm_blocks(0))
    for e in [one] + two:
        assert e.stats()["error"] == 0
        e.check_evaluator()
    for k, x in res.items():
        vs = sorted(v for v, _ in x)
        print(json.dumps({"arrangement": k, "median_exp_per_s": vs[len(vs) // 2], "min": vs[0], "max": vs[-1],
                          "ms_per_move": sorted(m for _, m in x)[len(x) // 2]}), flush=True)


if __name__ == "__main__":
    main()
