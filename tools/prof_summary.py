"""Summarise a rocprofv3 --kernel-trace --stats run into a small markdown table.

    python tools/prof_summary.py gpurun_out/prof/run_kernel_stats.csv [forwards] > profiles/x.md
"""
import csv
import sys


def short(name):
    n = name.replace("(anonymous namespace)::", "").split("(")[0]
    return n if len(n) < 70 else n[:67] + "..."


def main():
    path = sys.argv[1]
    forwards = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"source: `{path}`  (rocprofv3 --kernel-trace --stats)\n")
    print("| kernel | calls | total ms | avg us | % |")
    print("|---|---:|---:|---:|---:|")
    for r in rows[:25]:
        print(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['TotalDurationNs'])/1e6:.2f} | "
              f"{float(r['AverageNs'])/1e3:.1f} | {float(r['Percentage']):.2f} |")
    print(f"\nall kernels: {tot/1e6:.1f} ms")
    if forwards:
        nn = sum(float(r["TotalDurationNs"]) for r in rows
                 if not r["Name"].startswith("azg::") and "rocclr" not in r["Name"])
        conv = sum(float(r["TotalDurationNs"]) for r in rows if r["Name"].startswith("igemm_fwd"))
        tree = sum(float(r["TotalDurationNs"]) for r in rows
                   if r["Name"].startswith("azg::select") or r["Name"].startswith("azg::expand"))
        print(f"\nper forward ({forwards} forwards): network kernels {nn/forwards/1e6:.3f} ms, "
              f"igemm conv kernels {conv/forwards/1e6:.3f} ms, select+expand_backup {tree/forwards/1e3:.1f} us")


if __name__ == "__main__":
    main()
