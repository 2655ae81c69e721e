"""Device timeline of a rocprofv3 --kernel-trace run: per search cycle (the span
between consecutive launches of the anchor kernel), the time some kernel is
executing (union of intervals), the idle gaps and the kernels around them.

usage: python scripts/diag/timeline.py DIR/…kernel_trace.csv [anchor] [skip] [cycles]
(skip anchor launches at the start, then take `cycles` cycles; default: skip at
both ends)
"""
import csv
import sys
from collections import defaultdict


def short(name):
    n = name
    for pre in ("void ", "slamhip::", "(anonymous namespace)::"):
        n = n.replace(pre, "")
    return n.split("(")[0].split("<")[0]


def main():
    path = sys.argv[1]
    anchor = sys.argv[2] if len(sys.argv) > 2 else "sift_desc_band"
    skip = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    cycles = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    anchors = [r[0] for r in rows if r[2] == anchor]
    if len(anchors) < 2 * skip + 2:
        print("too few anchors", len(anchors))
        return
    if cycles:
        lo, hi, ncyc = anchors[skip], anchors[skip + cycles], cycles
    else:
        lo, hi = anchors[skip], anchors[-skip - 1]
        ncyc = len(anchors) - 2 * skip - 1
    sel = [r for r in rows if r[1] > lo and r[0] < hi]
    busy, gaps, cur_end, prev_name = 0, [], lo, None
    per = defaultdict(float)
    for s, e, n in sel:
        s2, e2 = max(s, lo), min(e, hi)
        per[n] += (e2 - s2) / 1e6
        if s2 > cur_end:
            gaps.append((s2 - cur_end, prev_name, n))
        if e2 > cur_end:
            busy += e2 - max(s2, cur_end)
            cur_end = e2
            prev_name = n
    span = (hi - lo) / 1e6
    print(f"cycles {ncyc}  span {span:.3f} ms  per cycle {span / ncyc:.3f} ms  busy {busy / 1e6 / ncyc:.3f} ms "
          f"({busy / 1e6 / span:.1%})  idle {(span - busy / 1e6) / ncyc:.3f} ms")
    print("kernel ms per cycle (sum of durations, overlaps counted twice):")
    for n, v in sorted(per.items(), key=lambda x: -x[1]):
        print(f"  {n:32s} {v / ncyc:.3f}")
    agg = defaultdict(lambda: [0, 0.0])
    for g, a, b in gaps:
        agg[(a, b)][0] += 1
        agg[(a, b)][1] += g / 1e6
    print("idle gaps by (before -> after): count, ms per cycle")
    for (a, b), (c, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:12]:
        print(f"  {a} -> {b}: {c}, {t / ncyc:.4f}")


if __name__ == "__main__":
    main()
