"""Summarise rocprofv3 PMC csv passes: mean counter value per kernel name (+ dispatch count)."""
import collections
import csv
import glob
import sys

root = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        if "wgk::" not in name and "k_" not in name:
            continue
        short = name.split("(")[0].replace("void ", "")
        acc[(short, r["Grid_Size"], r["LDS_Block_Size"], r["VGPR_Count"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} n={len(v):3d} mean={sum(v)/len(v):.4g}")
