#!/usr/bin/env python3
"""Sum rocprofv3 --pmc counter_collection CSVs per kernel (diagnostic).

    python tools/pmc_sum.py DIR [LABEL]   -> one JSON line {label, kernels: {name: {counter: sum}}}
"""
import csv
import glob
import json
import os
import re
import sys

d = sys.argv[1]
label = sys.argv[2] if len(sys.argv) > 2 else os.path.basename(d.rstrip("/"))
out = {}
for path in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
    for row in csv.DictReader(open(path)):
        name = row.get("Kernel_Name", "").replace("(anonymous namespace)::", "")
        name = re.sub(r"\(.*", "", name)
        name = re.sub(r"^(void )?([A-Za-z_0-9]+::)*", "", name)
        k = out.setdefault(name, {})
        k[row["Counter_Name"]] = k.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
print(json.dumps({"label": label, "kernels": out}))
