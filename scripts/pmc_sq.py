"""Mean SQ counter values per dispatch of the kernels whose name matches a
pattern, from a rocprofv3 --pmc run's counter_collection.csv.

    python3 scripts/pmc_sq.py <dir> [k_rows]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else "k_rows"
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    sums = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if pat not in k:
            continue
        k = k.split("(")[0]
        sums[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    out = {k: {c: v / len(disp[k]) for c, v in cs.items()} | {"dispatches": len(disp[k])}
           for k, cs in sums.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
