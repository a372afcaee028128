#!/usr/bin/env python3
"""HBM/fabric traffic per launch of the hot kernels from rocprofv3 PMC passes.

usage: python profiles/pmc_traffic.py <fetch counter_collection.csv> <write counter_collection.csv> [out.json [run]]
(run: the tag of the gpurun step the passes came from, stored as "_run" and quoted by bench.py)

Per MI355X_MICROARCH.md (HBM section): FETCH_SIZE (kB) counts the L2's
memory-side read requests and reports half the bytes of wide streaming reads
on gfx950, so it is doubled; WRITE_SIZE (kB) is taken as is.  The x2 holds for the 8
bytes-per-lane partner gathers too: one FETCH_SIZE pass over
tests/hip/gather_bench (16.13 GB of 112-wide f64 rows gathered per launch)
reads 7.85 GB, ratio 2.05 (profiles/r02_pmc_gather_calibration.txt).  Counters come from separate
--pmc passes (never combined with other tracing domains).  Launches are keyed
like bench.py's roofline kernel: "<user|item>_half/<kind>".
"""
import csv
import json
import re
import sys
from collections import defaultdict

# kernel symbol -> bench key ("<user|item>_half/gres_stage" for the streaming launch of each half)


def per_dispatch(path, counter):
    out = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        d = int(r["Dispatch_Id"])
        out[d] = (r["Kernel_Name"], out.get(d, (None, 0.0))[1] + float(r["Counter_Value"]))
    return out


def key_of(name, order_side):
    m = re.search(r"k_gres<(double|float), (\d+), (\d)(, \d+)?>", name)  # the streaming kernel (+ prefetch vectors)
    if m:
        return ("item" if m.group(3) == "1" else "user") + "_half/gres_stage"
    # Gram-block bins are several launches each (one per waves-per-row group, and the
    # f64 5-8-wave rows as 16-vector waves), so a per-launch figure does not match a
    # bin: only the streaming launches (one per half, the dominant kernel) are keyed
    return None


def main():
    fetch = per_dispatch(sys.argv[1], "FETCH_SIZE")
    write = per_dispatch(sys.argv[2], "WRITE_SIZE")
    out_path = sys.argv[3] if len(sys.argv) > 3 else None
    # a half's streaming rows may take two launches (f64 items: 8-wave tasks for rows up
    # to 1024 ratings, 16-wave ones above): a key's bytes are summed per sweep (sweeps
    # end at k_test) and averaged over the sweeps
    acc = {}
    for src, scale, field in ((fetch, 2.0, "fetch"), (write, 1.0, "write")):
        side = "user"
        sweep = 0
        for d in sorted(src):
            name, kb = src[d]
            if "k_gstream" in name or "k_gres" in name:  # a half's streaming launch precedes its gblock bins
                side = "item" if re.search(r"(k_gstream<\w+, \d+, \d+, \w+|k_gres<\w+, \d+), 1[,>]", name) else "user"
            if "k_test" in name:
                side = "user"
                sweep += 1
            k = key_of(name, side)
            if k is None:
                continue
            per = acc.setdefault(k, {"fetch": defaultdict(float), "write": defaultdict(float)})[field]
            per[sweep] += kb * 1024.0 * scale
    res = {}
    for k, v in acc.items():
        f = sum(v["fetch"].values()) / max(1, len(v["fetch"]))
        w = sum(v["write"].values()) / max(1, len(v["write"]))
        res[k] = f + w
    res["_note"] = ("bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (kB x 1024), averaged over the profiled "
                    "sweeps; x2 per MI355X_MICROARCH.md gfx950 note, checked for these 8 B/lane gathers on "
                    "tests/hip/gather_bench (ratio 2.05, r02_pmc_gather_calibration.txt)")
    if len(sys.argv) > 4:
        res["_run"] = sys.argv[4]
    txt = json.dumps(res, indent=1, sort_keys=True)
    print(txt)
    if out_path:
        open(out_path, "w").write(txt + "\n")


if __name__ == "__main__":
    main()
