"""Summarise rocprofv3 --pmc CSVs per kernel (average per dispatch) — used for profiles/*/pmc_summary.json."""
import collections
import csv
import json
import sys
from pathlib import Path


def summarise(paths, kernel_substr="loglik_kernel"):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for p in paths:
        for r in csv.DictReader(open(p)):
            if kernel_substr not in r["Kernel_Name"]:
                continue
            k = r["Kernel_Name"].split("(")[0]
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[(k, Path(p).name)].add(r["Dispatch_Id"])
    out = {}
    for k, d in agg.items():
        out[k] = {}
        for c, v in d.items():
            n = max(len(s) for (kk, _), s in disp.items() if kk == k)
            out[k][c] = v / n
    return out


if __name__ == "__main__":
    print(json.dumps(summarise(sys.argv[1:]), indent=1))
