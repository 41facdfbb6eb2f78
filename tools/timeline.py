"""Per-step kernel timeline from a rocprofv3 kernel trace (``--kernel-trace`` CSV).

Prints, for the last ``--steps`` occurrences of the step's anchor kernel, every kernel's start /
end relative to the step start (us) and its queue, plus the idle time in which no kernel ran:
shows how the graph branches of a split step overlap and where the GPU waits.

    python tools/timeline.py gpurun_out/x/prof/run_kernel_trace.csv [--anchor tail_adam] [--steps 3]
"""
import argparse
import csv


def short(name):
    n = name.split("(")[0]
    for key in ("jet_fwd_bf3_kernel", "jet_bwd_bf3_kernel"):
        if key in n:
            return key.replace("_kernel", "") + ("<x3>" if "Lb1E" in n or "true>" in n else "")
    return n[:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--anchor", default="tail_adam", help="kernel that ends a step")
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Queue_Id"]))
    rows.sort()
    ends = [i for i, r in enumerate(rows) if a.anchor in r[2]]
    if len(ends) < a.steps + 1:
        raise SystemExit(f"fewer than {a.steps + 1} '{a.anchor}' kernels in the trace")
    for k in range(len(ends) - a.steps, len(ends)):
        lo, hi = ends[k - 1] + 1, ends[k] + 1
        seg = rows[lo:hi]
        t0 = rows[ends[k - 1]][1]
        t_end = seg[-1][1]
        print(f"== step ending at dispatch {ends[k]}: {(t_end - t0) / 1e3:.1f} us from the previous step's end")
        busy, cur_s, cur_e = 0, None, None
        for s, e, n, q in seg:
            print(f"   q{q:>2} {(s - t0) / 1e3:8.1f} -> {(e - t0) / 1e3:8.1f}  ({(e - s) / 1e3:6.1f})  {short(n)}")
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        busy += cur_e - cur_s
        print(f"   busy {busy / 1e3:.1f} us, idle {(t_end - t0 - busy) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
