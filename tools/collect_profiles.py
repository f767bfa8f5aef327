#!/usr/bin/env python
"""Copy one GPU session's judged summaries (tools/gpu.sh <tag> ...) from
gpurun_out/<tag>/ into profiles/<round>/<name>/:

  rocprof_kernel_stats_{c3,16m,extra,c5}.csv   rocprofv3 --stats of the prof / roll5 steps
  pmc_traffic.json                             HBM bytes per launch from the FETCH_SIZE /
                                               WRITE_SIZE passes (MI355X_MICROARCH §HBM:
                                               2 x FETCH_SIZE + WRITE_SIZE, KiB), step and rollout
  bench_*.json, prof_*_bench.json, smoke.log, pytest_gpu_tail.txt, sq_rollout.txt

    python tools/collect_profiles.py <tag> profiles/r04/<name> [--build-info STR]

--build-info: the dd_build_info() of the library the session ran (the
pytest log's first line carries it; read from there when omitted).
"""
import argparse
import csv
import glob
import json
import os
import shutil

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def mean_counter(path, kernel, name):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == name]
    return (sum(vals) / len(vals), len(vals)) if vals else (None, 0)


def traffic(src, prefix, kernel):
    """{"fetch_bytes", "write_bytes", "bytes", "launches"} of one FETCH / WRITE pass pair."""
    fp = glob.glob(os.path.join(src, f"{prefix}FETCH_SIZE*", "*counter_collection.csv"))
    wp = glob.glob(os.path.join(src, f"{prefix}WRITE_SIZE*", "*counter_collection.csv"))
    if not fp or not wp:
        return None
    f, nf = mean_counter(fp[0], kernel, "FETCH_SIZE")
    w, nw = mean_counter(wp[0], kernel, "WRITE_SIZE")
    if f is None or w is None:
        return None
    return {"fetch_bytes": 2 * f * 1024, "write_bytes": w * 1024, "bytes": 2 * f * 1024 + w * 1024,
            "launches": [nf, nw]}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("tag")
    p.add_argument("dest")
    p.add_argument("--build-info", default="")
    a = p.parse_args()
    src = os.path.join(REPO, "gpurun_out", a.tag)
    dst = os.path.join(REPO, a.dest)
    os.makedirs(dst, exist_ok=True)
    info = a.build_info
    log = os.path.join(src, "pytest_gpu.log")
    if os.path.exists(log):
        lines = open(log).read().splitlines()
        if not info and lines and "build_info:" in lines[0]:
            info = lines[0].split("build_info:", 1)[1].split(";md5")[0].split("; md5")[0].strip()
        with open(os.path.join(dst, "pytest_gpu_tail.txt"), "w") as f:
            f.write("\n".join(lines[:1] + lines[-3:]) + "\n")
    for name in ("c3", "16m", "extra", "c5", "k20"):
        hits = glob.glob(os.path.join(src, f"prof_{name}", "*kernel_stats.csv"))
        if hits:
            shutil.copy(hits[0], os.path.join(dst, f"rocprof_kernel_stats_{name}.csv"))
    for pat in ("bench_*.json", "prof_*_bench.json", "smoke.log", "*.jsonl", "*trace_summary.json",
                "*summary.json"):
        for f in glob.glob(os.path.join(src, pat)):
            shutil.copy(f, dst)
    rows = {}
    for n in (262144, 16777216):
        t = None
        fp = glob.glob(os.path.join(src, f"pmc_FETCH_SIZE_{n}", "*counter_collection.csv"))
        wp = glob.glob(os.path.join(src, f"pmc_WRITE_SIZE_{n}", "*counter_collection.csv"))
        if fp and wp:
            f, nf = mean_counter(fp[0], "step_kernel", "FETCH_SIZE")
            w, nw = mean_counter(wp[0], "step_kernel", "WRITE_SIZE")
            t = {"fetch_bytes": 2 * f * 1024, "write_bytes": w * 1024, "bytes": 2 * f * 1024 + w * 1024,
                 "algorithmic_bytes": 147 * n, "launches": [nf, nw]}
        if t:
            rows[f"step_{n}"] = t
    r = traffic(src, "pmc_roll_", "rollout_kernel")
    if r:
        r["workload"] = "config 5: 65,536 drones x 256 frames, one dd_rollout launch (tools/prof_driver.py)"
        rows["rollout_65536x256"] = r
    if rows:
        json.dump({"build_info": info, "rows": rows, "formula": "2*FETCH_SIZE*1024 + WRITE_SIZE*1024 per launch"},
                  open(os.path.join(dst, "pmc_traffic.json"), "w"), indent=1)
    sq = os.path.join(REPO, "gpurun_out", f"{a.tag}_sqroll.log")
    if os.path.exists(sq):
        shutil.copy(sq, os.path.join(dst, "sq_rollout.txt"))
    print(json.dumps({"dest": a.dest, "build_info": info, "files": sorted(os.listdir(dst))}))


if __name__ == "__main__":
    main()
