"""Summarise a rocprofv3 --kernel-trace --stats run from its rocpd database
(ROCm 7.2's default output) into the markdown table tools/prof_summary.py makes
from the CSV.

    python tools/prof_db_summary.py gpurun_out/<dir>/run_results.db > profiles/x.md
"""
import sqlite3
import sys


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    return n if len(n) < 70 else n[:67] + "..."


def main():
    path = sys.argv[1]
    c = sqlite3.connect(path)
    rows = list(c.execute("select name, total_calls, total_duration, average, percentage from top_kernels"))
    rows.sort(key=lambda r: -float(r[2]))
    tot = sum(float(r[2]) for r in rows)
    print(f"source: `{path}`  (rocprofv3 --kernel-trace --stats; durations in the db are us)\n")
    print("| kernel | calls | total ms | avg us | % |")
    print("|---|---:|---:|---:|---:|")
    for name, calls, total, avg, pct in rows[:25]:
        print(f"| `{short(name)}` | {calls} | {float(total) / 1e3:.2f} | {float(avg):.1f} | {float(pct):.2f} |")
    print(f"\nall kernels: {tot / 1e3:.1f} ms")


if __name__ == "__main__":
    main()
