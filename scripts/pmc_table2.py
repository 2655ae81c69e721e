"""Per-kernel average of every counter in rocprofv3 --pmc passes (largest grid only).
usage: python scripts/pmc_table2.py DIR1 [DIR2 ...]"""
import collections
import csv
import glob
import re
import sys

vals = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = re.split(r"[<(]", r["Kernel_Name"].replace("slamhip::(anonymous namespace)::", "").replace("void ", ""))[0]
            vals[k][r["Counter_Name"]].append((int(r["Grid_Size"]), float(r["Counter_Value"])))
for k, cs in vals.items():
    print(k)
    for c, v in sorted(cs.items()):
        g = max(x[0] for x in v)
        xs = [x[1] for x in v if x[0] == g]
        print(f"   {c:28s} {sum(xs) / len(xs):16.4g}   (n={len(xs)}, grid={g})")
