"""Per-kernel duration percentiles from a rocprofv3 kernel-trace CSV: kdist.py trace.csv prefix..."""
import csv
import sys

import numpy as np


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    for k in sys.argv[2:]:
        v = np.array([(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
                      for r in rows if r["Kernel_Name"].startswith(k)])
        if len(v):
            print(f"{k:28s} n={len(v):5d} mean {v.mean():7.2f}  p0/10/50/90/100 "
                  + " ".join(f"{x:7.2f}" for x in np.percentile(v, [0, 10, 50, 90, 100])))


if __name__ == "__main__":
    main()
