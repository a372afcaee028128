"""Per-sweep device timeline from a rocprofv3 CSV run (kernel trace, optional memory-copy and HIP
API traces): python3 timeline.py <dir-with-csvs> [sweeps]

A sweep starts at each launch of the user half's first streaming kernel (k_gres<...,0>, the
first one after a non-user launch).  For the last `sweeps` sweeps it prints every device
operation (kernel or copy) with its start offset, duration and the idle gap before it (union of
busy intervals), then the per-sweep span / busy / idle, and the host API calls that overlap the
largest idle gaps."""
import csv
import glob
import os
import re
import sys


def rows(d, pat):
    f = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


def short(n):
    n = n.replace("sbmf::(anonymous namespace)::", "").replace("void ", "")
    n = re.sub(r"\(.*", "", n)
    return n[:60]


def main():
    d = sys.argv[1]
    want = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    ops = []
    for r in rows(d, "*kernel_trace.csv"):
        ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K", short(r["Kernel_Name"]), r.get("Stream_Id", "")))
    for r in rows(d, "*memory_copy_trace.csv"):
        ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C", r.get("Direction", "copy"), ""))
    ops.sort()
    api = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]) for r in rows(d, "*hip_api_trace.csv")]
    api.sort()
    user = [i for i, o in enumerate(ops) if o[2] == "K" and re.search(r"k_gres<[^>]*, ?0>", o[3])]
    # the learner with the most sweeps (a bench run also holds a short serial-schedule learner)
    streams = [ops[i][4] for i in user]
    main_s = max(set(streams), key=streams.count)
    user = [i for i in user if ops[i][4] == main_s]
    starts, seen_item = [], True
    for i, o in enumerate(ops):  # the first user streaming launch after an item one
        if o[2] != "K" or o[4] != main_s:
            continue
        if re.search(r"k_gres<[^>]*, ?1>", o[3]):
            seen_item = True
        elif seen_item and re.search(r"k_gres<[^>]*, ?0>", o[3]):
            starts.append(i)
            seen_item = False
    # a sweep = from one user-half streaming start to the next (windows far above the median
    # span hold another leg's work: dropped)
    if len(starts) < 2:
        print("no sweeps found")
        return
    pairs = list(zip(starts[:-1], starts[1:]))
    spans = sorted(ops[b][0] - ops[a][0] for a, b in pairs)
    med = spans[len(spans) // 2]
    sel = [p for p in pairs if ops[p[1]][0] - ops[p[0]][0] < 2 * med][-want:]
    tot_span = tot_idle = 0.0
    for a, b in sel:
        t0 = ops[a][0]
        t1 = ops[b][0]
        busy_end = t0
        idle = 0
        gaps = []
        print("---- sweep window %.1f us" % ((t1 - t0) / 1e3))
        for o in ops[a:b]:
            gap = max(0, o[0] - busy_end)
            if gap:
                gaps.append((gap, busy_end, o[0]))
            idle += gap
            busy_end = max(busy_end, o[1])
            print("  %8.1f  %7.1f  gap %6.1f  %s %s s%s" % ((o[0] - t0) / 1e3, (o[1] - o[0]) / 1e3, gap / 1e3, o[2], o[3], o[4]))
        idle += max(0, t1 - busy_end)
        if t1 > busy_end:
            gaps.append((t1 - busy_end, busy_end, t1))
        span = t1 - t0
        tot_span += span
        tot_idle += idle
        print("  span %.1f us, idle %.1f us (%.0f %%)" % (span / 1e3, idle / 1e3, 100.0 * idle / span))
        for g, s, e in sorted(gaps, reverse=True)[:3]:
            calls = [x for x in api if x[1] > s and x[0] < e]
            print("  gap %.1f us at %.1f: host calls in it: %s" % (
                g / 1e3, (s - t0) / 1e3,
                ", ".join("%s %.1f" % (x[2], (x[1] - x[0]) / 1e3) for x in calls[:12])))
    print("mean span %.1f us, idle %.1f us (%.0f %%)" % (tot_span / len(sel) / 1e3, tot_idle / len(sel) / 1e3,
                                                        100.0 * tot_idle / tot_span))


if __name__ == "__main__":
    main()
