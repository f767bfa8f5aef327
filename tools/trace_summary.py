#!/usr/bin/env python
"""Per-launch durations of one kernel from a rocprofv3 kernel trace (and, for
a counter-collection CSV, the effective clock GRBM_GUI_ACTIVE / 8 / duration
per dispatch), with the averages over all launches and over the last N — the
launches bench.py times after its warm ones (rollout_point: 1 + 120 warm, 40
timed).

    python tools/trace_summary.py TRACE.csv --kernel rollout_kernel --last 40

--grid N keeps the launches of N lanes (Grid_Size_X) and --slice A:B the
launches A..B-1 of those (in dispatch order): the driver-shaped bench line's
20 timed config-3 steps are --grid 262144 --slice 8:28 (3 settle launches and
the 5 warm-up steps come first).
"""
import argparse
import csv
import json
import re
import statistics


def main():
    p = argparse.ArgumentParser()
    p.add_argument("csv")
    p.add_argument("--kernel", default="rollout_kernel")
    p.add_argument("--last", type=int, default=40)
    p.add_argument("--grid", type=int, default=0, help="only launches of this many lanes (Grid_Size_X)")
    p.add_argument("--slice", default="", help="A:B, launches A..B-1 of the selected ones")
    args = p.parse_args()
    rows = [r for r in csv.DictReader(open(args.csv)) if re.search(args.kernel, r["Kernel_Name"])
            and (not args.grid or int(r.get("Grid_Size_X", 0)) == args.grid)]
    per = {}
    for r in rows:
        d = per.setdefault(int(r["Dispatch_Id"]), {"us": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3,
                                                   "t0": int(r["Start_Timestamp"]), "t1": int(r["End_Timestamp"]),
                                                   "kernel": r["Kernel_Name"]})
        if "Counter_Name" in r:
            d[r["Counter_Name"]] = float(r["Counter_Value"])
    ids = sorted(per)
    if args.slice:
        a, b = (int(x) if x else None for x in args.slice.split(":"))
        ids = ids[a:b]
    us = [per[i]["us"] for i in ids]
    out = {"source": args.csv, "kernel_regex": args.kernel, "grid": args.grid or None, "slice": args.slice or None, "kernels": sorted({per[i]["kernel"] for i in ids}),
           "launches": len(us), "us_mean_all": round(statistics.mean(us), 2),
           "last": args.last, "us_mean_last": round(statistics.mean(us[-args.last:]), 2),
           "us_median_last": round(statistics.median(us[-args.last:]), 2),
           "us_per_launch": [round(u, 1) for u in us]}
    if len(ids) > 1:  # idle time between one selected launch's end and the next one's start
        gaps = [(per[b]["t0"] - per[a]["t1"]) / 1e3 for a, b in zip(ids, ids[1:])]
        out["gap_us_median"] = round(statistics.median(gaps), 2)
        out["span_us"] = round((per[ids[-1]]["t1"] - per[ids[0]]["t0"]) / 1e3, 2)
    if ids and "GRBM_GUI_ACTIVE" in per[ids[0]]:
        ghz = [per[i]["GRBM_GUI_ACTIVE"] / 8 / (per[i]["us"] * 1e3) for i in ids]
        out["effective_clock_ghz"] = [round(g, 3) for g in ghz]
        out["shader_kcycles_per_launch"] = [round(g * u, 1) for g, u in zip(ghz, us)]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
