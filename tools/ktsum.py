"""Per-kernel summary of rocprofv3 --kernel-trace CSVs: python tools/ktsum.py DIR [DIR...]"""
import collections
import csv
import glob
import os
import sys

for d in sys.argv[1:]:
    acc = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            acc[r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][-40:]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(f"== {d}")
    for k, x in sorted(acc.items(), key=lambda kv: -sum(kv[1]))[:30]:
        print(f"  {k:42s} {len(x):5d} {sum(x) / len(x):10.1f} us avg {sum(x):10.1f} us")
