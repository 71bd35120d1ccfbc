#!/usr/bin/env python3
"""Summarise tools/pmc_util.sh's counter pass: per learner kernel, the mean over launches of
each counter and the effective clock GRBM_GUI_ACTIVE / 8 / duration (MI355X_MICROARCH.md, DVFS:
rocprofv3 sums GRBM over the 8 XCDs).  usage: tools/pmc_util.py <dir with run_counter_collection.csv>"""
import collections, csv, os, sys

root = sys.argv[1]
f = [os.path.join(d, x) for d, _, fs in os.walk(root) for x in fs if x.endswith("counter_collection.csv")][0]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
dur = {}
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:48]
    disp = r.get("Dispatch_Id", r.get("Correlation_Id", ""))
    vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    if "End_Timestamp" in r and "Start_Timestamp" in r:
        dur.setdefault(k, {})[disp] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
names = ["GRBM_GUI_ACTIVE", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES",
         "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE"]
print(f"{'kernel':48s} " + " ".join(f"{n[:16]:>16s}" for n in names) + "   us   GHz  lds_conf/active")
for k, c in sorted(vals.items(), key=lambda kv: -sum(kv[1].get("SQ_WAVE_CYCLES", [0]))):
    m = {n: (sum(c[n]) / len(c[n]) if c.get(n) else float("nan")) for n in names}
    d = dur.get(k, {})
    us = sum(d.values()) / len(d) if d else float("nan")
    ghz = m["GRBM_GUI_ACTIVE"] / 8 / (us * 1e3) if us == us and us > 0 else float("nan")
    lc = m["SQ_LDS_BANK_CONFLICT"] / m["SQ_LDS_IDX_ACTIVE"] if m["SQ_LDS_IDX_ACTIVE"] else float("nan")
    print(f"{k:48s} " + " ".join(f"{m[n]:16.4g}" for n in names) + f" {us:6.2f} {ghz:5.2f} {lc:8.3f}")
