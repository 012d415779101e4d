"""Per-kernel counter values per launch (averaged over launches) from rocprofv3 --pmc CSV output.
usage: python tools/pmc_dump.py <dir> [kernel-substring]"""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
per = defaultdict(lambda: defaultdict(float))
n = defaultdict(set)
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for row in csv.DictReader(fh):
            name = (row.get("Kernel_Name") or "").replace("(anonymous namespace)::", "").replace("void ", "")
            if flt not in name:
                continue
            key = name.split("(")[0]
            per[key][row["Counter_Name"]] += float(row["Counter_Value"])
            n[key].add(row.get("Dispatch_Id") or row.get("Correlation_Id"))
for k, c in sorted(per.items()):
    m = max(1, len(n[k]))
    print(f"{k}  ({m} launches)")
    for cn, v in sorted(c.items()):
        print(f"   {cn:32s} {v / m:16.1f}")
