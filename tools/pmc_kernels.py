"""Per-kernel mean of any rocprofv3 PMC counters (one or more counter_collection.csv
files of separate passes): value per dispatch summed over its rows, averaged over the
kernel's dispatches.  Usage: python tools/pmc_kernels.py [--match SUBSTR] a.csv [b.csv ...]"""
import csv
import sys
from collections import defaultdict


def main():
    args = sys.argv[1:]
    match = ""
    if args and args[0] == "--match":
        match, args = args[1], args[2:]
    per = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))   # kernel -> counter -> dispatch -> value
    for path in args:
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"]
            if match and match not in k:
                continue
            per[k][r["Counter_Name"]][(path, r.get("Dispatch_Id", ""))] += float(r["Counter_Value"])
    for k, cs in sorted(per.items()):
        print(k[:150])
        for c, d in sorted(cs.items()):
            v = list(d.values())
            print(f"   {c:32s} {sum(v) / len(v):16.1f}   ({len(v)} dispatches)")


if __name__ == "__main__":
    main()
