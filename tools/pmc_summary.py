"""Summarise rocprofv3 --pmc CSVs under gpurun_out/pmc: per-counter mean per dispatch for the kernel regex."""
import csv
import glob
import re
import sys
from collections import defaultdict

regex = re.compile(sys.argv[1] if len(sys.argv) > 1 else "fwd_f16")
root = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out/pmc"
vals = defaultdict(list)
for f in sorted(glob.glob(f"{root}/p*/**/*counter_collection.csv", recursive=True)):
    with open(f) as fh:
        for row in csv.DictReader(fh):
            if not regex.search(row.get("Kernel_Name", "")):
                continue
            vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
for k in sorted(vals):
    v = vals[k]
    print(f"{k:32s} n={len(v):3d} mean={sum(v)/len(v):.6g}")
