#!/usr/bin/env python3
"""HBM/fabric traffic of online VB's factor passes per epoch, from rocprofv3 PMC passes.

usage: python profiles/pmc_vb.py <fetch counter_collection.csv> <write counter_collection.csv> [out.json [run]]

The factor passes are every mini-batch's 2K launches of k_user_v and k_item_vp (plus k_item_v,
the sliced items' update) in vbo.hip -- the epoch's dominant kernels, which bench.py's online-VB
line times with HIP events (sbmf_timing.ms_vb_factor).  Bytes = 2 x FETCH_SIZE + WRITE_SIZE
(kB x 1024), the gfx950 correction of pmc_traffic.py; summed over the profiled run and divided by
its epochs (one vbo k_test launch per epoch).
"""
import csv
import json
import re
import sys

FACTOR = re.compile(r"::(k_user_v<|k_item_vp<|k_item_v\()")


def per_dispatch(path, counter):
    out = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        d = int(r["Dispatch_Id"])
        out[d] = (r["Kernel_Name"], out.get(d, (None, 0.0))[1] + float(r["Counter_Value"]))
    return out


def main():
    fetch = per_dispatch(sys.argv[1], "FETCH_SIZE")
    write = per_dispatch(sys.argv[2], "WRITE_SIZE")
    res = {}
    for src, scale, field in ((fetch, 2.0, "fetch"), (write, 1.0, "write")):
        epochs = sum(1 for n, _ in src.values() if re.search(r"::k_test\(", n))
        tot = sum(kb for n, kb in src.values() if FACTOR.search(n)) * 1024.0 * scale
        res[field] = tot / max(1, epochs)
        res["epochs_" + field] = epochs
    out = {"vb_factor_passes": res["fetch"] + res["write"], "epochs_profiled": res["epochs_fetch"],
           "_note": "bytes per epoch of the factor passes (k_user_v, k_item_vp, k_item_v) = 2 x FETCH_SIZE + "
                    "WRITE_SIZE (kB x 1024), averaged over the profiled epochs"}
    if len(sys.argv) > 4:
        out["_run"] = sys.argv[4]
    txt = json.dumps(out, indent=1, sort_keys=True)
    print(txt)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(txt + "\n")


if __name__ == "__main__":
    main()
