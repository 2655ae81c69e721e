"""BA kernel-trace summary of the last solve in a rocprofv3 --kernel-trace csv
(scripts/ba_prof.sh): span, kernel-busy time, launches, per-kernel averages.
usage: python scripts/ba_kt.py gpurun_out/TAG_w8 [gpurun_out/TAG_w16 ...]"""
import csv
import glob
import re
import sys
from collections import defaultdict


def summary(d):
    rows = list(csv.DictReader(open(glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0])))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows
                 if "ba_" in r["Kernel_Name"]))
    first = max(i for i, k in enumerate(ks) if "ba_eval_init" in k[2])
    ks = ks[first:]
    span = (ks[-1][1] - ks[0][0]) / 1e6
    busy = sum(e - s for s, e, _ in ks) / 1e6
    print(f"{d} last solve: span ms {span:.3f} kernel busy ms {busy:.3f} launches {len(ks)}")
    agg = defaultdict(list)
    for s, e, n in ks:
        agg[re.search(r"(ba_\w+)", n).group(1)].append((e - s) / 1e3)
    for n, v in sorted(agg.items(), key=lambda x: -sum(x[1])):
        print(f"   {n:30s} {sum(v) / 1e3:6.3f} ms  n={len(v):4d}  avg {sum(v) / len(v):7.2f} us")


for d in sys.argv[1:]:
    summary(d)
