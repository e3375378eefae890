"""Summarise rocprofv3 --pmc CSVs (one dir per pass) into per-kernel averages."""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

out = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for row in csv.DictReader(fh):
            name = row.get("Kernel_Name", "?")
            m = re.search(r"(\w+)<[^()]*>\(", name) or re.search(r"(\w+)\(", name)
            short = m.group(1) if m else name
            acc[short][row["Counter_Name"]].append(float(row["Counter_Value"]))
res = {}
for k, d in acc.items():
    res[k] = {c: sum(v) / len(v) for c, v in d.items()}
    res[k]["_dispatches_per_counter"] = {c: len(v) for c, v in d.items()}
print(json.dumps(res, indent=1))
