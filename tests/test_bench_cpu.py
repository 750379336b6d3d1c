"""bench.py's algorithmic byte and FLOP models (no GPU): the per-leaf figures DESIGN.md
quotes and the roofline fields are priced with."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402


def test_direct_net_flops_match_survey():
    total, conv234 = bench.net_flops(7, 4, 343)
    assert round(total / 1e6, 1) == 404.3 and round(conv234 / 1e6, 1) == 391.6


def test_winograd_gemm_flops():
    # (11^2 + 7^2 + 5^2) transformed points x 2 x 512^2 per leaf
    assert bench.winograd_flops(7) == (121 + 49 + 25) * 2 * 512 * 512


def test_transform_bytes():
    tb = bench.transform_bytes(7, 4)
    assert tb["first"] == 4 * 49 * 4 + 121 * 512 * 4
    assert tb["mid"] == (121 + 49) * 512 * 4 + (49 + 25) * 512 * 4
    assert tb["out"] == 25 * 512 * 4 + 9 * 512 * 6
    assert tb["total"] == tb["first"] + tb["mid"] + tb["out"] == 827152


def test_tree_bytes_per_expansion():
    # ~4.8 KB per expansion at d = 1.33, A = 87
    b = bench.tree_bytes_per_exp(343, 4 * 49 * 4)
    assert 4700 < b < 4800


def test_committed_pmc_traffic():
    """The committed round-5 PMC pass the bench line's `traffic` fields and games/s HBM roofline read:
    the split GEMM near its algorithmic ~0.91 GB per launch (4 launches per forward), a whole
    simulation step at 4096 leaves between the GEMMs + transforms and 10 GB."""
    pmc = bench.load_pmc(4096, "inflexion", "winograd")
    assert pmc is not None
    assert 3.4e9 < pmc["split_gemm_per_forward"] < 4.2e9
    assert 3.0e9 < pmc["transforms"] < 3.8e9
    assert pmc["split_gemm_per_forward"] + pmc["transforms"] < pmc["step_total"] < 10e9
    assert bench.load_pmc(256, "inflexion", "winograd") is None  # measured at G = 4096 only


def test_presets_are_the_baseline_configs():
    assert bench.PRESETS["C4"] == dict(game="inflexion", n=7, games=4096, sims=25)
    assert bench.PRESETS["C2"]["games"] == 256 and bench.PRESETS["C3"]["sims"] == 100
    assert bench.PRESETS["C5"] == dict(game="othello", n=8, games=4096, sims=200)


def test_gpus_n_launches_n_ranks():
    """`bench.py --gpus 2` with no launcher env starts 2 ranks (a child torchrun) with
    RANK / LOCAL_RANK / WORLD_SIZE set; each rank stops before any GPU call here."""
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR",
                                                             "MASTER_PORT")}
    out = subprocess.run([sys.executable, bench.__file__, "--gpus", "2", "--print-rank-env"], env=env,
                         capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [json.loads(x) for x in out.stdout.splitlines() if x.startswith("{")]
    assert sorted((d["rank"], d["local_rank"], d["world_size"]) for d in lines) == [(0, 0, 2), (1, 1, 2)]
    assert all(d["master_addr"] == "127.0.0.1" and d["gpus"] == 2 for d in lines)


def test_rank_command_is_the_drivers_form():
    cmd = bench.rank_command(8, ["--gpus", "8", "--steps", "3"], 29500)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--master-addr" in cmd and "127.0.0.1" in cmd
    assert cmd[-4:] == ["--gpus", "8", "--steps", "3"]


def test_cpu_baseline_core_count():
    usable, machine = bench.host_cores()
    assert 1 <= usable <= machine


def test_cpu_worker_runs_a_bounded_sample():
    """One single-threaded cpu_baseline worker (what each of the per-core processes runs)."""
    import json
    import subprocess
    out = subprocess.run([sys.executable, bench.__file__, "--cpu-worker", "3", "--cpu-proc-moves", "1"],
                         capture_output=True, text=True, timeout=300, env=dict(os.environ, OMP_NUM_THREADS="1"))
    assert out.returncode == 0, out.stderr[-2000:]
    d = json.loads(out.stdout.strip().splitlines()[-1])
    assert d["moves"] == 1 and 1 <= d["expansions"] <= 25 and d["seconds"] > 0
