"""Summarise rocprofv3 --pmc CSVs (one directory per pass) into per-kernel averages."""
import csv
import glob
import json
import sys
from collections import defaultdict


def load(root):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(f"{root}/p*/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
            acc[r["Kernel_Name"]]["_vgpr"] = [float(r["VGPR_Count"])]
            acc[r["Kernel_Name"]]["_lds"] = [float(r["LDS_Block_Size"])]
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in acc.items()}


if __name__ == "__main__":
    res = load(sys.argv[1])
    for k, d in sorted(res.items()):
        print(k)
        for c, v in sorted(d.items()):
            print(f"   {c:28s} {v:16.1f}")
    if len(sys.argv) > 2:
        json.dump(res, open(sys.argv[2], "w"), indent=1)
