"""Per-step kernel timeline from a rocprofv3 ``--kernel-trace`` SQLite database (``run_results.db``):
for the last ``--steps`` steps (ending at the ``--anchor`` kernel), every kernel's start / end relative
to the previous anchor's end (us) and its hardware queue - where the step's branches overlap and
where the GPU idles.

    python tools/timeline_db.py gpurun_out/<run>/prof/run_results.db [--anchor tail_adam] [--steps 3]
"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--anchor", default="tail_adam")
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = list(c.execute("select name, start, end, queue_id from kernels order by start"))
    idx = [i for i, r in enumerate(rows) if r[0].startswith(a.anchor)]
    for n, k in enumerate(idx[-a.steps:]):
        j = idx[idx.index(k) - 1]
        t0 = rows[j][2]
        print(f"--- step (anchor end -> anchor end {(rows[k][2] - t0) / 1e3:.2f} us)")
        for r in rows[j + 1:k + 1]:
            print(f"{(r[1] - t0) / 1e3:8.2f} {(r[2] - t0) / 1e3:8.2f}  q{r[3]}  {r[0].split('(')[0][:60]}")


if __name__ == "__main__":
    main()
