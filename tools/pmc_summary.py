"""Average rocprofv3 --pmc counters per kernel name over the passes of tools/pmc_kernel.sh."""
import collections
import csv
import glob
import os
import sys


def main(d):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "")
            name = (name[5:] if name.startswith("void ") else name).split("(")[0][:70]
            acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for name, cs in acc.items():
        print(name)
        for c, v in sorted(cs.items()):
            print(f"   {c:28s} {sum(v) / len(v):16.4g}   (n={len(v)})")


if __name__ == "__main__":
    main(sys.argv[1])
