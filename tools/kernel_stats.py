"""Per-step kernel table from a rocprofv3 ``--kernel-trace --stats --output-format csv`` run.

    python tools/kernel_stats.py gpurun_out/<run>/prof/run_kernel_stats.csv --steps 55 [--title ...]

Prints ``us_per_step calls pct kernel`` rows sorted by time (the format of profiles/*_kernel_stats.txt).
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=int, required=True, help="profiled optimizer steps (warmup + timed)")
    ap.add_argument("--title", default="")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    if a.title:
        print(f"# {a.title}")
    print("# us_per_step  calls  pct  kernel")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[: a.top]:
        ns = float(r["TotalDurationNs"])
        print(f"{ns / 1e3 / a.steps:9.1f} {int(r['Calls']):6d} {100 * ns / tot:5.1f}%  {r['Name'][:150]}")
    print(f"# total {tot / 1e6 / a.steps:.3f} ms/step (profiled)")


if __name__ == "__main__":
    main()
