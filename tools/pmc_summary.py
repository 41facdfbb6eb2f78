"""Per-kernel PMC summary of a tools/gpu_runs/r2_pmc.sh run: python tools/pmc_summary.py gpurun_out/<run>

Prints per-dispatch averages and per-wave figures (cycles: SQ_WAVE_CYCLES / WAIT_* / ACTIVE_* count
quad-cycles on gfx950 and are scaled x4 here; SQ_VALU_MFMA_BUSY_CYCLES counts cycles)."""
import collections
import csv
import glob
import sys


def main():
    root = sys.argv[1]
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.defaultdict(int)
    for f in sorted(glob.glob(f"{root}/pmc*/**/*counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")
            k = k.split("(")[0][:48]
            key = (k, r["Counter_Name"])
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            cnt[key] += 1
    for k, d in agg.items():
        print(f"== {k}")
        waves = d.get("SQ_WAVES", 0) / max(1, cnt[(k, "SQ_WAVES")])
        for c, v in sorted(d.items()):
            per = v / max(1, cnt[(k, c)])
            quad = c in ("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                         "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_LDS",
                         "SQ_ACTIVE_INST_MISC", "SQ_ACTIVE_INST_SCA", "SQ_WAIT_INST_LDS")
            pw = per * (4 if quad else 1) / waves if waves and c != "SQ_WAVES" else float("nan")
            print(f"   {c:28s} {per:12.4g}   per wave {pw:10.4g}")


if __name__ == "__main__":
    main()
