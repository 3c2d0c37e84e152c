"""Per-kernel averages of every PMC counter under a directory of rocprofv3 --pmc runs.
    python tools/pmc_summary.py <dir> [kernel-substring ...]"""
import collections
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    want = sys.argv[2:]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
        with open(path) as f:
            for row in csv.DictReader(f):
                name = row["Kernel_Name"].split("(")[0]
                if want and not any(w in name for w in want):
                    continue
                acc[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for name, cs in sorted(acc.items()):
        print(name)
        for c, v in sorted(cs.items()):
            print(f"    {c:28s} {sum(v) / len(v):18.1f}  (n={len(v)})")


if __name__ == "__main__":
    main()
