"""Summarise rocprofv3 --pmc csv outputs: per kernel name, mean counter value per dispatch."""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for row in csv.DictReader(fh):
            name = row.get("Kernel_Name", "?")
            short = name.split("(")[0].replace("void ", "")[:60]
            acc[short][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, cs in acc.items():
    print(k)
    for c, vals in sorted(cs.items()):
        print(f"   {c:28s} {sum(vals) / len(vals):16.1f}  (n={len(vals)})")
