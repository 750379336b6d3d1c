"""Per-launch view of one kernel in a rocprofv3 --kernel-trace run: its duration distribution, the
kernel that ran before it on the queue, the gap since that kernel ended, and its duration split by
predecessor -- to tell a kernel's own cost from what the stream around it does to it (VERDICT r04
item 6: winograd_first at 192 us in the engine against 175-179 us timed alone).

    python tools/trace_summary.py gpurun_out/x/trace/run_kernel_trace.csv winograd_first > profiles/y.json
"""
import csv
import json
import statistics
import sys


def short(name):
    n = name.replace("(anonymous namespace)::", "").split("(")[0]
    return n if len(n) < 60 else n[:57] + "..."


def main():
    path, pat = sys.argv[1], sys.argv[2]
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    out = {"source": path, "kernel": pat, "launches": 0}
    durs, gaps, by_prev = [], [], {}
    for i, r in enumerate(rows):
        if pat not in r["Kernel_Name"]:
            continue
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        durs.append(d)
        if i:
            p = rows[i - 1]
            gaps.append((int(r["Start_Timestamp"]) - int(p["End_Timestamp"])) / 1e3)
            by_prev.setdefault(short(p["Kernel_Name"]), []).append(d)
    if durs:
        durs_sorted = sorted(durs)
        out.update(launches=len(durs), mean_us=statistics.mean(durs), median_us=statistics.median(durs),
                   p10_us=durs_sorted[len(durs) // 10], p90_us=durs_sorted[9 * len(durs) // 10],
                   min_us=durs_sorted[0], max_us=durs_sorted[-1],
                   gap_after_previous_us={"mean": statistics.mean(gaps) if gaps else None,
                                          "median": statistics.median(gaps) if gaps else None},
                   by_previous_kernel={k: {"launches": len(v), "mean_us": statistics.mean(v)}
                                       for k, v in sorted(by_prev.items(), key=lambda kv: -len(kv[1]))},
                   first_10_us=durs[:10])
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
