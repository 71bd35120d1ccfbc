#!/usr/bin/env python3
"""Per-kernel table of the counters collected by tools/pmc.sh (mean per dispatch)."""
import collections, csv, glob, os, sys
sys.path.insert(0, os.path.dirname(__file__))
from summarize_profile import short

root = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(root, "p*", "run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        vals[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
cols = sys.argv[2].split(",") if len(sys.argv) > 2 else sorted({c for k in vals for c in vals[k]})
print("kernel".ljust(14) + "".join(c[-14:].rjust(15) for c in cols))
for k, d in sorted(vals.items()):
    if k.startswith("void") or k.startswith("__"):
        continue
    print(k[:14].ljust(14) + "".join((f"{sum(d[c]) / len(d[c]):15.4g}" if d.get(c) else " " * 15) for c in cols))
