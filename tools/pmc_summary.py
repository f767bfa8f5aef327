#!/usr/bin/env python
"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of the step kernel
into profiles/pmc_traffic.json (read by bench.py for roofline.traffic).

Per MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are KiB; on gfx950
FETCH_SIZE counts each 128-B fabric read request as 64 B, so the read bytes
are 2 x FETCH_SIZE x 1024; WRITE_SIZE x 1024 are the written bytes.  The two
counters come from separate passes (FETCH_SIZE needs 3 TCC slots, WRITE_SIZE 2).

    python tools/pmc_summary.py OUT.json [--rollout FRAMES] ENVS PRECISION OBS FETCH.csv WRITE.csv [...]

(--rollout FRAMES: the passes are of dd_rollout launches of FRAMES frames, rollout_kernel rows)

Each row records the library's dd_build_info() (ABI version + step-kernel ISA
hash) of the build the passes ran on — the in-tree libdronestep.so, which is
what travels to the GPU box — so bench.py can refuse counters of another build.
"""
import csv
import json
import sys


def mean_counter(path, name, kernel="step_kernel"):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == name]
    if not vals:
        raise SystemExit(f"no {name} rows for {kernel} in {path}")
    return sum(vals) / len(vals), len(vals)


def build_info() -> str:
    import os
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(repo, "reinforcement-learning-101_amd"))
    from delivery_drone_amd import abi
    return abi.lib().dd_build_info().decode()


def main():
    out = sys.argv[1]
    info = build_info()
    args = sys.argv[2:]
    kernel, frames = "step_kernel", None
    if args[:1] == ["--rollout"]:  # --rollout FRAMES: rows of dd_rollout launches of FRAMES frames
        kernel, frames, args = "rollout_kernel", int(args[1]), args[2:]
    try:
        doc = json.load(open(out))
    except (OSError, ValueError):
        doc = {"note": __doc__.strip().splitlines()[0], "rows": []}
    for i in range(0, len(args), 5):
        envs, prec, obs, fpath, wpath = args[i:i + 5]
        fetch, nf = mean_counter(fpath, "FETCH_SIZE", kernel)
        write, nw = mean_counter(wpath, "WRITE_SIZE", kernel)
        row = {"envs": int(envs), "precision": prec, "obs": obs == "1",
               "fetch_size_kib": round(fetch, 3), "write_size_kib": round(write, 3),
               "read_bytes_per_launch": int(2 * fetch * 1024), "write_bytes_per_launch": int(write * 1024),
               "hbm_bytes_per_launch": int(2 * fetch * 1024 + write * 1024), "dispatches": [nf, nw],
               "source": [fpath, wpath], "build_info": info}
        if kernel != "step_kernel":
            row.update(kernel=kernel, frames=frames)
        doc["rows"] = [r for r in doc["rows"] if not (r["envs"] == row["envs"] and r["precision"] == prec
                                                      and r["obs"] == row["obs"]
                                                      and r.get("kernel", "step_kernel") == kernel
                                                      and r.get("frames") == frames)] + [row]
    json.dump(doc, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
