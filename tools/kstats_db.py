"""Per-step kernel table from a rocprofv3 ``--kernel-trace`` SQLite database (``run_results.db``).

    python tools/kstats_db.py gpurun_out/<run>/prof/run_results.db --steps 60

Prints ``us_per_step calls avg_us kernel`` rows sorted by total time (the format of
profiles/*_kernel_stats.txt; tools/kernel_stats.py reads the CSV output instead).
"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, required=True, help="profiled optimizer steps (warmup + timed)")
    ap.add_argument("--top", type=int, default=20)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = list(c.execute("select name, count(*), avg(duration), sum(duration) from kernels group by name "
                          "order by sum(duration) desc"))
    tot = sum(r[3] for r in rows)
    print("# us_per_step  calls  avg_us  pct  kernel")
    for name, n, avg, s in rows[:a.top]:
        print(f"{s / 1e3 / a.steps:9.1f} {n:7d} {avg / 1e3:8.2f} {100 * s / tot:5.1f}%  {name[:120]}")
    print(f"# total {tot / 1e6 / a.steps:.3f} ms/step (profiled)")


if __name__ == "__main__":
    main()
