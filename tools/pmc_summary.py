#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter CSVs for the geodesic kernel (per dispatch, summed over XCDs/SEs)."""
import collections
import csv
import glob
import json
import sys


def summarise(root, kernel="sr_integrate_kernel<true, false"):
    out = {}
    for p in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
        agg = collections.defaultdict(float)
        disp = collections.defaultdict(set)
        for r in csv.DictReader(open(p)):
            if kernel not in r.get("Kernel_Name", ""):
                continue
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            disp[r["Counter_Name"]].add(r["Dispatch_Id"])
        for c, v in agg.items():
            out[c] = v / max(1, len(disp[c]))
    return out


if __name__ == "__main__":
    for root in sys.argv[1:]:
        print(root, json.dumps({k: f"{v:.4g}" for k, v in sorted(summarise(root).items())}, indent=0))
