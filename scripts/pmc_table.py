"""Print per-kernel averages of rocprofv3 counter passes (gpurun_out/TAG_p*/).
usage: python scripts/pmc_table.py TAG [KERNEL_SUBSTR]"""
import collections, csv, glob, os, re, sys

tag = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else ""
base = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gpurun_out")
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(base, f"{tag}_p*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = re.split(r"[<(]", r["Kernel_Name"].replace("slamhip::(anonymous namespace)::", "").replace("void ", ""))[0]
        if sub in k:
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"  {c:28s} {sum(v) / len(v):16.4g}  (n={len(v)})")
