#!/usr/bin/env python3
"""LDS bank-conflict share per launch of the hot kernels from a rocprofv3
--pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS pass (profiles/collect.sh lds).

usage: python profiles/pmc_lds.py <counter_collection.csv> [out.json [run]]
conflict_per_active = SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS: the cycles the
LDS pipe stalls on bank conflicts per cycle spent issuing LDS instructions,
summed over every SIMD of the launch and averaged over the profiled sweeps;
frac = SQ_LDS_BANK_CONFLICT / (SQ_LDS_BANK_CONFLICT + SQ_ACTIVE_INST_LDS): the
share of the LDS pipe's cycles lost to conflicts (bench.py's
roofline.lds_bank_conflict_frac).  Keys as
bench.py's roofline kernel ("<user|item>_half/<kind>").
"""
import csv
import json
import re
import sys
from collections import defaultdict

from pmc_traffic import key_of


def main():
    per = defaultdict(lambda: defaultdict(float))
    names = {}
    for r in csv.DictReader(open(sys.argv[1])):
        d = int(r["Dispatch_Id"])
        per[d][r["Counter_Name"]] += float(r["Counter_Value"])
        names[d] = r["Kernel_Name"]
    acc = defaultdict(lambda: [0.0, 0.0, 0.0, 0])
    side = "user"
    for d in sorted(per):
        name = names[d]
        if "k_gstream" in name or "k_gres" in name:
            side = "item" if re.search(r"(k_gstream<\w+, \d+, \d+, \w+|k_gres<\w+, \d+), 1[,>]", name) else "user"
        if "k_test" in name:
            side = "user"
        k = key_of(name, side)
        if not k:
            continue
        a = acc[k]
        a[0] += per[d].get("SQ_LDS_BANK_CONFLICT", 0.0)
        a[1] += per[d].get("SQ_ACTIVE_INST_LDS", 0.0)
        a[2] += per[d].get("SQ_INSTS_LDS", 0.0)
        a[3] += 1
    out = {"_note": "conflict_per_active = SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS, frac = SQ_LDS_BANK_CONFLICT / "
                    "(SQ_LDS_BANK_CONFLICT + SQ_ACTIVE_INST_LDS), per launch (rocprofv3 --pmc, profiles/collect.sh lds)"}
    for k, (bc, act, ins, n) in sorted(acc.items()):
        out[k] = {"bank_conflict_cycles": bc / n, "lds_active_cycles": act / n, "lds_insts": ins / n,
                  "conflict_per_active": bc / act if act else None,
                  "frac": bc / (bc + act) if bc + act else None}
    if len(sys.argv) > 3:
        out["_run"] = sys.argv[3]  # the gpurun step the pass came from (quoted by bench.py)
    s = json.dumps(out, indent=1)
    print(s)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(s + "\n")


if __name__ == "__main__":
    main()
