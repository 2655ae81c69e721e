"""Per-launch SQ counters of one kernel family from rocprofv3 --pmc passes.

usage: python scripts/diag/pmc_sum.py REGEX DIR [DIR ...]
Each DIR is a rocprofv3 -d output (run_counter_collection.csv); the counters of
every dispatch whose kernel name matches REGEX are summed over the dispatches
and divided by their count, then a few ratios are derived (per-XCD cycles:
GRBM_GUI_ACTIVE / 8; 1024 SIMDs).
"""
import csv
import re
import sys
from collections import defaultdict


def main():
    rx = re.compile(sys.argv[1])
    tot = defaultdict(float)
    disp = defaultdict(set)
    for d in sys.argv[2:]:
        with open(f"{d}/run_counter_collection.csv") as f:
            for r in csv.DictReader(f):
                if not rx.search(r["Kernel_Name"]):
                    continue
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
                disp[r["Counter_Name"]].add((d, r["Dispatch_Id"]))
    per = {k: v / len(disp[k]) for k, v in tot.items()}
    out = {k: f"{v:.4g}" for k, v in sorted(per.items())}
    g = per.get("GRBM_GUI_ACTIVE")
    if g:
        cyc = g / 8
        simd = 1024 * cyc
        for k, name in (("SQ_ACTIVE_INST_VALU", "valu_active_frac"), ("SQ_ACTIVE_INST_LDS", "lds_inst_active_frac"),
                        ("SQ_ACTIVE_INST_SCA", "salu_active_frac")):
            if k in per:
                out[name] = round(per[k] / simd * 4, 3)    # SQ_ACTIVE_INST_* count per SIMD in units of 4 cycles
        if "SQ_LDS_IDX_ACTIVE" in per:
            out["lds_idx_active_frac"] = round(per["SQ_LDS_IDX_ACTIVE"] / (256 * cyc), 3)
        if "SQ_INSTS_VALU" in per:
            out["valu_issue_frac_2cyc"] = round(per["SQ_INSTS_VALU"] * 2 / simd, 3)
        if "SQ_LDS_BANK_CONFLICT" in per and "SQ_LDS_IDX_ACTIVE" in per:
            out["lds_conflict_frac"] = round(per["SQ_LDS_BANK_CONFLICT"] / max(per["SQ_LDS_IDX_ACTIVE"], 1), 4)
        out["kernel_ms_at_2.4GHz"] = round(cyc / 2.4e6, 3)
    print(out)


if __name__ == "__main__":
    main()
