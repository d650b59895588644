"""Summarise scripts/probe/red_pmc.sh output: per-dispatch averages of every counter of
the reduce kernel, per pass directory."""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/red_pmc"
for d in sorted(glob.glob(f"{root}/p*")):
    tot, cnt = defaultdict(float), defaultdict(set)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "reduce_kernel" not in r.get("Kernel_Name", ""):
                continue
            k = r["Counter_Name"]
            tot[k] += float(r["Counter_Value"])
            cnt[k].add(r["Dispatch_Id"])
    print(d, {k: round(tot[k] / max(len(cnt[k]), 1), 1) for k in sorted(tot)})
