"""First move at which the batched engine's trace leaves the reference's, per seed, for one golden set
over several (gemm form, G) -- which leaf-batch shapes / evaluator paths reproduce a set exactly.

    python tools/realnet_sweep.py peaked_sims100 split:4096 split:2048 split:1024 f32:4096
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_lib as ol  # noqa: E402
import test_gpu_realnet as tr  # noqa: E402


def run(name, gemm, G):
    from azg_amd.engine import SelfPlayEngine
    from azg_amd.nnet import InferenceNet
    data = ol.load_json(f"mcts_{name}.json.gz")
    cfg, eps = data["config"], data["episodes"]
    kind, n, _ = tr.SETS[name]
    net = tr._ref_net(kind, n, name)
    e = SelfPlayEngine(G, sims=cfg["sims"], cpuct=cfg["cpuct"], temp_threshold=cfg["temp_threshold"],
                       max_turns=cfg.get("max_turns", 343), seed_base=0, first_game=eps[0]["seed"],
                       evaluator=InferenceNet(net, gemm=gemm), game=kind, n=n)
    e.play()
    st = e.stats()
    rec = e.read_moves()
    out = {}
    for i, ep in enumerate(eps):
        A = rec["counts"][i].shape[-1]
        m = tr._first_mismatch(ep["moves"], rec["counts"][i], rec["actions"][i], int(rec["moves"][i]), 0, A)
        out[ep["seed"]] = m
    e.close()
    return {"set": name, "gemm": gemm, "G": G, "first_mismatch": out, "error": st["error"],
            "max_live_nodes": st.get("max_live_nodes"), "max_depth": st.get("max_depth")}


def main():
    import azg_amd  # noqa: F401
    name = sys.argv[1]
    for spec in sys.argv[2:]:
        gemm, G = spec.split(":")
        print(json.dumps(run(name, gemm, int(G))), flush=True)


if __name__ == "__main__":
    main()
