"""Average rocprofv3 --pmc counters per kernel family: python tools/pmc_table.py <dir> [<dir> ...]"""
import collections
import csv
import glob
import os
import re
import sys


def family(name):
    m = re.match(r"(?:void )?(?:krcn::)?(k_\w+)", name)
    base = m.group(1) if m else name[:40]
    for tag in ("EpiSlicePart", "EpiLz2", "EpiLz1", "EpiHvpOut", "EpiWeighted", "EpiStore", "EpiGrad"):
        if tag in name:
            return f"{base}<{tag}>"
    return base


def main():
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in sys.argv[1:]:
        for f in glob.glob(os.path.join(d, "**", "*_counter_collection.csv"), recursive=True):
            per = collections.defaultdict(lambda: collections.defaultdict(float))
            for r in csv.DictReader(open(f)):
                key = (r["Kernel_Name"], r.get("Dispatch_Id", r.get("Correlation_Id", "")))
                per[key][r["Counter_Name"]] += float(r["Counter_Value"])
            for (name, _), cs in per.items():
                for c, v in cs.items():
                    acc[family(name)][c].append(v)
    for fam, cs in sorted(acc.items()):
        print(fam)
        for c, vs in sorted(cs.items()):
            print(f"    {c:40s} {sum(vs) / len(vs):16.1f}  (n={len(vs)})")


if __name__ == "__main__":
    main()
