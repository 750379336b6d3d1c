"""Evaluator accuracy on the peaked-prior network (tests/golden peaked_net: the trained network's fc3 x 16)
at the root positions of its reference traces: P (relative error over valid actions, by prior size) and v
of each GPU form -- the split form at 4096 and 256 leaves, the f32-GEMM form, the small-batch path --
against the reference module on the CPU (batch 1, f32; what NNetWrapper.predict computes).

    python tools/peaked_diag.py > gpurun_out/peaked_diag.json
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import azg_amd  # noqa: E402,F401
import oracle_lib as ol  # noqa: E402
from azg_amd.flags import PlayerColour  # noqa: E402
from azg_amd.inflexion import InflexionGame  # noqa: E402
from azg_amd.nnet import InferenceNet, InflexionNNet  # noqa: E402


def positions(name, seeds, every):
    d = ol.load_json(f"mcts_{name}.json.gz")
    g0 = InflexionGame(7, max_turns=d["config"]["max_turns"], max_power=6)
    out = []
    for ep in d["episodes"]:
        if ep["seed"] not in seeds:
            continue
        for m, mv in enumerate(ep["moves"]):
            if m % every and m not in seeds[ep["seed"]]:
                continue
            g = g0.restarted()
            g._board = np.asarray(mv["board"]).reshape(7, 7).astype(g._board.dtype)
            g._curr_turn = mv["turn"]
            g._player = PlayerColour.RED if mv["turn"] % 2 == 0 else PlayerColour.BLUE
            out.append((ep["seed"], m, g.to_planes(), g.valid_actions_mask().astype(bool)))
    return out


def main():
    torch.manual_seed(0)
    cpu = ol.peaked_net(InflexionNNet()).eval()
    gpu = ol.peaked_net(InflexionNNet()).cuda().eval()
    pos = positions("peaked_main", {7: {320, 321, 322, 323}, 3: {305}, 1: {307}}, 40) + \
        positions("peaked_sims100", {10: {0, 1, 2, 3, 4, 5, 6}, 11: set()}, 10)
    x = torch.tensor(np.array([p[2] for p in pos]), dtype=torch.float32)
    with torch.no_grad():
        lp, v_ref = cpu(x)
    p_ref = torch.exp(lp).numpy().astype(np.float64)
    v_ref = v_ref.numpy().reshape(-1).astype(np.float64)
    forms = {"split": InferenceNet(gpu, gemm="split"), "f32": InferenceNet(gpu, gemm="f32"),
             "module": None}
    res = {}
    for fname, ev in forms.items():
        for B in ((4096, 256) if fname == "split" else (1024,) if fname == "f32" else (len(pos),)):
            xb = x.cuda()
            if B > len(pos):
                xb = torch.cat([xb, xb[:1].expand(B - len(pos), -1, -1, -1)])
            with torch.no_grad():
                if ev is None:
                    lpg, vg = gpu(xb)
                    pg = torch.exp(lpg)
                else:
                    pg, vg = ev(xb)
            pg = pg[:len(pos)].double().cpu().numpy()
            vg = vg.reshape(-1)[:len(pos)].double().cpu().numpy()
            rows = []
            for i, (seed, m, _, valid) in enumerate(pos):
                pr, pgi = p_ref[i][valid], pg[i][valid]
                big = pr > 1e-6
                tiny = (pr > 0) & (pr <= 1e-6)
                rows.append({"seed": seed, "move": m,
                             "max_rel_p_big": float(np.max(np.abs(pgi[big] - pr[big]) / pr[big])) if big.any() else 0.0,
                             "max_rel_p_tiny": float(np.max(np.abs(pgi[tiny] - pr[tiny]) / pr[tiny])) if tiny.any() else 0.0,
                             "zero_mismatch": int(np.sum((pr == 0) != (pgi == 0))),
                             "order_mismatch": int(np.sum(np.argsort(-pr, kind="stable")[:8] != np.argsort(-pgi, kind="stable")[:8])),
                             "abs_v": float(abs(vg[i] - v_ref[i])), "v": float(v_ref[i]),
                             "max_p": float(pr.max())})
            worst = {k: max(r[k] for r in rows) for k in ("max_rel_p_big", "max_rel_p_tiny", "zero_mismatch",
                                                          "order_mismatch", "abs_v")}
            res[f"{fname}@{B}"] = {"worst": worst,
                                   "focus": [r for r in rows if (r["seed"], r["move"]) in
                                             {(7, 322), (10, 5), (10, 4), (1, 307), (3, 305)}]}
            print(json.dumps({"form": f"{fname}@{B}", **res[f"{fname}@{B}"]}), flush=True)


def mixed():
    """Every GPU form on a realistic leaf batch: 4096 distinct positions from the golden traces (all
    three networks' games), each form's P / v against the CPU module at batch 1, worst and 99.9th
    percentile per form (the split form's operand scales are batch-wide: a mixed batch is the case
    the engine runs)."""
    torch.manual_seed(0)
    cpu = ol.peaked_net(InflexionNNet()).eval()
    gpu = ol.peaked_net(InflexionNNet()).cuda().eval()
    pos = []
    for name in ("peaked_main", "trained_main", "realnet_main", "peaked_sims100"):
        pos += positions(name, {s: set() for s in range(200)}, 1)
    rs = np.random.RandomState(0)
    pos = [pos[i] for i in rs.permutation(len(pos))[:4096]]
    x = torch.tensor(np.array([p[2] for p in pos]), dtype=torch.float32)
    valid = np.array([p[3] for p in pos])
    with torch.no_grad():
        ref = [cpu(x[i:i + 1]) for i in range(len(pos))]
    p_ref = np.concatenate([torch.exp(r[0]).numpy() for r in ref]).astype(np.float64)
    v_ref = np.concatenate([r[1].numpy().reshape(-1) for r in ref]).astype(np.float64)
    ev_split, ev_f32 = InferenceNet(gpu, gemm="split"), InferenceNet(gpu, gemm="f32")
    for fname, ev, B in (("split", ev_split, 4096), ("split", ev_split, 256), ("split", ev_split, 512),
                         ("f32", ev_f32, 1024), ("module", None, 4096)):
        pg, vg = [], []
        with torch.no_grad():
            for i in range(0, len(pos), B):
                xb = x[i:i + B].cuda()
                if ev is None:
                    a, b = gpu(xb)
                    a = torch.exp(a)
                else:
                    a, b = ev(xb)
                pg.append(a.double().cpu().numpy())
                vg.append(b.reshape(-1).double().cpu().numpy())
        pg, vg = np.concatenate(pg), np.concatenate(vg)
        rel = np.where(valid & (p_ref > 1e-6), np.abs(pg - p_ref) / np.maximum(p_ref, 1e-300), 0).max(axis=1)
        relt = np.where(valid & (p_ref > 0) & (p_ref <= 1e-6), np.abs(pg - p_ref) / np.maximum(p_ref, 1e-300),
                        0).max(axis=1)
        av = np.abs(vg - v_ref)
        worst = int(np.argmax(rel))
        print(json.dumps({"mixed": f"{fname}@{B}", "rel_p_big_max": float(rel.max()),
                          "rel_p_big_p999": float(np.quantile(rel, 0.999)), "rel_p_big_median": float(np.median(rel)),
                          "rel_p_tiny_max": float(relt.max()), "abs_v_max": float(av.max()),
                          "abs_v_p999": float(np.quantile(av, 0.999)),
                          "worst": {"slot": worst, "seed": pos[worst][0], "move": pos[worst][1]}}), flush=True)


def leaves():
    """The reference's own leaves (tests/golden/peaked_leaves_*.npz: planes as predict got them, its P
    and v) through every GPU form: log-space prior error per leaf, zero / nonzero disagreements, v."""
    torch.manual_seed(0)
    gpu = ol.peaked_net(InflexionNNet()).cuda().eval()
    d = np.load(os.path.join(ROOT, "tests", "golden", "peaked_leaves_peaked_sims100_s10.npz"))
    x = torch.tensor(d["x"].astype(np.float32))
    p_ref, v_ref, mv = d["p"].astype(np.float64), d["v"].astype(np.float64), d["move"]
    n = len(x)
    for fname, B in (("split", 1024), ("split", 512), ("split", 256), ("f32", 1024), ("module", 1)):
        ev = None if fname == "module" else InferenceNet(gpu, gemm=fname)
        pg, vg = [], []
        with torch.no_grad():
            for i in range(0, n, B):
                xb = x[i:i + B].cuda()
                k = xb.shape[0]
                if k < B:
                    xb = torch.cat([xb, xb[:1].expand(B - k, -1, -1, -1)])
                if ev is None:
                    a, b = gpu(xb)
                    a = torch.exp(a)
                else:
                    a, b = ev(xb)
                pg.append(a[:k].double().cpu().numpy())
                vg.append(b.reshape(-1)[:k].double().cpu().numpy())
        pg, vg = np.concatenate(pg), np.concatenate(vg)
        both = (p_ref > 1e-38) & (pg > 1e-38)
        lerr = np.where(both, np.abs(np.log(np.where(both, pg, 1)) - np.log(np.where(both, p_ref, 1))), 0).max(axis=1)
        zero = ((p_ref == 0) != (pg == 0)).sum(axis=1)
        sub = ((p_ref > 0) & (p_ref < 1.2e-38) & (pg != p_ref)).sum(axis=1)
        verr = np.abs(vg - v_ref)
        order = np.argsort(-lerr)[:5]
        print(json.dumps({"leaves": f"{fname}@{B}", "n": n, "log_err_max": float(lerr.max()),
                          "log_err_p99": float(np.quantile(lerr, 0.99)), "n_log_err_gt_1e-4": int((lerr > 1e-4).sum()),
                          "zero_mismatch_leaves": int((zero > 0).sum()), "subnormal_diff_leaves": int((sub > 0).sum()),
                          "v_err_max": float(verr.max()), "v_worst": int(np.argmax(verr)),
                          "worst": [[int(i), int(mv[i]), float(lerr[i])] for i in order]}), flush=True)


def engine_slot(G=1024, gemm="split", moves=7, slot=0):
    """The batched engine on peaked_sims100 (first game 10) with the evaluator wrapped: every leaf batch's
    row `slot` (planes, P, v) against the CPU module at batch 1 and the same form on a batch of copies."""
    import copy
    from azg_amd.engine import SelfPlayEngine
    torch.manual_seed(0)
    gpu = ol.peaked_net(InflexionNNet()).cuda().eval()
    cpu = copy.deepcopy(gpu).cpu()
    ev = InferenceNet(gpu, gemm=gemm)
    log = []

    class Rec:
        outputs_probs = True

        def __call__(self, planes):
            p, v = ev(planes)
            log.append((planes[slot].clone(), p[slot].clone(), v.reshape(-1)[slot].clone()))
            return p, v

        def check_range(self):
            ev.check_range()
    d = ol.load_json("mcts_peaked_sims100.json.gz")
    cfg = d["config"]
    e = SelfPlayEngine(G, sims=cfg["sims"], cpuct=cfg["cpuct"], temp_threshold=cfg["temp_threshold"],
                       max_turns=cfg["max_turns"], seed_base=0, first_game=10, evaluator=Rec(), game="inflexion", n=7)
    e.play(max_moves=moves)
    out = []
    for k, (x, p, v) in enumerate(log):
        xc = x.unsqueeze(0).cpu()
        with torch.no_grad():
            lp, vr = cpu(xc)
            pr = torch.exp(lp)[0].double().numpy()
            pc, vc = ev(x.unsqueeze(0).expand(G, -1, -1, -1).contiguous())
        pg = p.double().cpu().numpy()
        pc = pc[0].double().cpu().numpy()
        both = (pr > 1e-38) & (pg > 1e-38)
        lerr = float(np.max(np.where(both, np.abs(np.log(np.where(both, pg, 1)) - np.log(np.where(both, pr, 1))), 0)))
        diff_copy = float(np.max(np.abs(pg - pc)))
        out.append((k, lerr, float(abs(v.item() - vr.item())), diff_copy, float(abs(v.item() - vc.reshape(-1)[0].item()))))
    ref = np.load(os.path.join(ROOT, "tests", "golden", "peaked_leaves_peaked_sims100_s10.npz"))
    first = None
    maxerr = 0.0
    for k, (x, p, v) in enumerate(log[:len(ref["x"])]):
        if not np.array_equal(x.cpu().numpy().astype(np.int8), ref["x"][k]):
            first = k
            break
        pr, pg = ref["p"][k].astype(np.float64), p.double().cpu().numpy()
        both = (pr > 1e-38) & (pg > 1e-38)
        maxerr = max(maxerr, float(np.max(np.where(both, np.abs(np.log(np.where(both, pg, 1)) - np.log(np.where(both, pr, 1))), 0))))
    print(json.dumps({"engine_slot": f"{gemm}@{G}", "first_leaf_mismatch": first,
                      "move": int(ref["move"][first]) if first is not None else None,
                      "max_log_err_vs_reference_before": maxerr}), flush=True)
    if first is not None:
        for k in range(max(0, first - 3), first + 1):
            x, p, v = log[k]
            print(json.dumps({"k": k, "ref_v": float(ref["v"][k]), "eng_v": float(v.item()),
                              "same_planes": bool(np.array_equal(x.cpu().numpy().astype(np.int8), ref["x"][k]))}))
    worst = sorted(out, key=lambda t: -t[1])[:8]
    wv = sorted(out, key=lambda t: -t[2])[:5]
    comp = sorted(out, key=lambda t: -max(t[3], t[4]))[:5]
    print(json.dumps({"engine_slot": f"{gemm}@{G}", "calls": len(out), "worst_log_err": worst, "worst_v": wv,
                      "batch_dependence": comp}), flush=True)
    e.close()


if __name__ == "__main__":
    if "--engine" in sys.argv:
        engine_slot(1024, "split")
        engine_slot(512, "split")
        sys.exit(0)
    leaves() if "--leaves" in sys.argv else mixed() if "--mixed" in sys.argv else main()
