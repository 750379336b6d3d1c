"""HBM traffic per kernel from separate rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

    python tools/pmc_summary.py <fetch_counter_collection.csv> <write_counter_collection.csv> > profiles/x.json

Corrections per MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced streaming read,
so the read side is doubled (an upper-bound correction for kernels whose reads
are not all 16-B-per-lane streams).
"""
import csv
import json
import sys
from collections import defaultdict


def load(path, counter):
    """{(kernel name, grid size): [counter value per dispatch]}"""
    per = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name") != counter:
            continue
        per[(r["Kernel_Name"], int(r["Grid_Size"]))].append(float(r["Counter_Value"]))
    return per


def median(xs):
    xs = sorted(xs)
    return xs[len(xs) // 2] if xs else 0.0


def group(name):
    if name.startswith("igemm_fwd") and "bt128x128" in name:
        return "conv2-4 igemm"
    if name.startswith("igemm_fwd"):
        return "conv1 igemm"
    if "azg::select_kernel" in name:
        return "select_kernel"
    if "azg::expand_backup_kernel" in name:
        return "expand_backup_kernel"
    if "azg::expand_select_kernel" in name:
        return "expand_select_kernel"
    if "azg::move_end_kernel" in name:
        return "move_end_kernel"
    if "bias_relu" in name:
        return "bias_relu_nhwc"
    if "winograd_first" in name:
        return "winograd_first"
    if "winograd_mid" in name:
        return "winograd_mid"
    if "winograd_in" in name:
        return "winograd_in"
    if "winograd_out" in name:
        return "winograd_out"
    if "split_gemm_persist" in name:  # the 256-row persistent schedule: conv2-4, fc1 (bench's `roofline`)
        return "split_gemm"
    if "split_gemm" in name:  # 128 / 64-row schedules: fc2, [fc3 | fc4] at 4096 leaves
        return "split_gemm_small"
    if name.startswith("Cijk_"):
        return "gemm (hipBLASLt)"
    return None


def main():
    fetch = load(sys.argv[1], "FETCH_SIZE")
    write = load(sys.argv[2], "WRITE_SIZE")
    out = {}
    for key in sorted(set(fetch) | set(write), key=lambda k: (k[0], -k[1])):
        g = group(key[0])
        if g is None:
            continue
        f, w = fetch.get(key, []), write.get(key, [])
        out.setdefault(g, []).append({
            "grid": key[1], "dispatches": max(len(f), len(w)),
            "fetch_kib_raw_median": median(f), "write_kib_median": median(w),
            "fetch_bytes_corrected": 2 * median(f) * 1024, "write_bytes": median(w) * 1024,
            "hbm_bytes": 2 * median(f) * 1024 + median(w) * 1024})
    # per leaf forward = per simulation: totals over all dispatches / simulations (robust where
    # several layers share one kernel name and grid, e.g. the three GEMM batches).  A simulation
    # starts with select_kernel (a move's first) or expand_select_kernel (the previous one's
    # expand / backup fused with this one's select: azg_sim_end_begin)
    tot = defaultdict(lambda: [0.0, 0.0, 0])
    for key in set(fetch) | set(write):
        g = group(key[0])
        if g is None:
            continue
        tot[g][0] += 2 * sum(fetch.get(key, [])) * 1024
        tot[g][1] += sum(write.get(key, [])) * 1024
        tot[g][2] += max(len(fetch.get(key, [])), len(write.get(key, [])))
    n_fwd = sum(tot[g][2] for g in ("select_kernel", "expand_select_kernel") if g in tot)
    summary = {}
    for g, v in out.items():
        f, w, n = tot[g]
        summary[g] = {"per_shape": v, "hbm_bytes_sum_over_shapes": sum(x["hbm_bytes"] for x in v),
                      "dispatches": n, "fetch_bytes_corrected_total": f, "write_bytes_total": w,
                      "hbm_bytes_per_forward": (f + w) / n_fwd if n_fwd else None}
    summary["_forwards"] = n_fwd
    json.dump(summary, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
