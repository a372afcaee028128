#!/usr/bin/env python3
"""Per-kernel PMC summary of one Gibbs sweep from a rocprofv3 counter_collection.csv.

usage: python profiles/pmc_summary.py <counter_collection.csv> [--sweep -1]
Groups the rows of each dispatch, takes the dispatches of one sweep (between
two consecutive k_test launches; default the last complete one) and prints
kernel, grid, duration and every counter collected.  FETCH_SIZE is shown raw
(kB) and corrected x2 per MI355X_MICROARCH.md's gfx950 note.
"""
import csv
import re
import sys
from collections import OrderedDict


def short(name):
    m = re.search(r"(k_\w+)(<[^>(]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:40]


def load(path):
    disp = OrderedDict()
    for r in csv.DictReader(open(path)):
        d = disp.setdefault(int(r["Dispatch_Id"]), {"name": short(r["Kernel_Name"]), "grid": int(r["Grid_Size"]) // max(1, int(r["Workgroup_Size"])),
                                                     "wg": int(r["Workgroup_Size"]), "ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                                                     "c": OrderedDict()})
        d["c"][r["Counter_Name"]] = d["c"].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return list(disp.values())


def main():
    path = sys.argv[1]
    which = int(sys.argv[sys.argv.index("--sweep") + 1]) if "--sweep" in sys.argv else -1
    ds = load(path)
    tests = [i for i, d in enumerate(ds) if d["name"].startswith("k_test")]
    if len(tests) < 2:
        sel = ds
    else:
        pairs = list(zip(tests[:-1], tests[1:]))
        a, b = pairs[which]
        sel = ds[a + 1:b + 1]
    keys = []
    for d in sel:
        for k in d["c"]:
            if k not in keys:
                keys.append(k)
    print("counters: " + ", ".join(keys))
    print("%-34s %7s %4s %9s " % ("kernel", "grid", "wg", "us") + " ".join("%14s" % k[-14:] for k in keys))
    for d in sel:
        if d["ns"] < 20000:
            continue
        vals = []
        for k in keys:
            v = d["c"].get(k, float("nan"))
            vals.append("%14.4g" % v)
        print("%-34s %7d %4d %9.1f " % (d["name"][:34], d["grid"], d["wg"], d["ns"] / 1e3) + " ".join(vals))


if __name__ == "__main__":
    main()
