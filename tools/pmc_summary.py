#!/usr/bin/env python3
"""Fold a gpu_profile.sh run (gpurun_out/) into the committed profiles/ directory.

profiles/<round>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (bench command)
profiles/<round>_bench.json         the bench line measured in the same call
profiles/pmc_traffic.json           per-kernel HBM traffic per launch from the separate
                                    FETCH_SIZE / WRITE_SIZE passes, corrected as
                                    MI355X_MICROARCH.md (HBM section) prescribes:
                                    bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024
                                    (FETCH_SIZE is KiB and reads half of a wide streaming read
                                    on gfx950; WRITE_SIZE is KiB, exact for streaming stores)
usage: python tools/pmc_summary.py r01 [gpurun_out]
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_kernel(path, counter):
    acc = collections.defaultdict(list)
    for row in csv.DictReader(open(path)):
        if row["Counter_Name"] != counter:
            continue
        name = row["Kernel_Name"].split("(")[0].replace("void ", "").replace("skm::", "")
        acc[name].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    rnd = sys.argv[1]
    src = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "gpurun_out")
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "prof_trace", "run_kernel_stats.csv"), os.path.join(dst, f"{rnd}_kernel_stats.csv"))
    bench = json.load(open(os.path.join(src, "bench.json")))
    json.dump(bench, open(os.path.join(dst, f"{rnd}_bench.json"), "w"), indent=1)
    legs = os.path.join(src, "prof_trace_legs", "run_kernel_stats.csv")
    if os.path.exists(legs):
        shutil.copy(legs, os.path.join(dst, f"{rnd}_kernel_stats_legs.csv"))
    fetch = per_kernel(os.path.join(src, "prof_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(src, "prof_write", "run_counter_collection.csv"), "WRITE_SIZE")
    # kernels of the annotate / matrix legs from their own passes (the build kernels of those
    # passes also ran the matrix leg's smaller training build, so they are not taken from there)
    fl = os.path.join(src, "prof_fetch_legs", "run_counter_collection.csv")
    if os.path.exists(fl):
        f2 = per_kernel(fl, "FETCH_SIZE")
        w2 = per_kernel(os.path.join(src, "prof_write_legs", "run_counter_collection.csv"), "WRITE_SIZE")
        for k in set(f2) | set(w2):
            if k not in fetch and k not in write:
                fetch[k] = f2.get(k, 0.0)
                write[k] = w2.get(k, 0.0)
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        f, w = fetch.get(k, 0.0), write.get(k, 0.0)
        kernels[k] = {"FETCH_SIZE_KiB": f, "WRITE_SIZE_KiB": w,
                      "hbm_bytes_per_launch": (2.0 * f + w) * 1024.0}
    out = {"round": rnd, "seqs_per_gpu": bench["config"]["seqs_per_gpu"],
           "formula": "(2*FETCH_SIZE + WRITE_SIZE) * 1024 bytes per launch (gfx950 FETCH_SIZE correction)",
           "note": "FETCH_SIZE counts Infinity-Cache hits too, so gathers served on-die are included",
           "kernels": kernels}
    json.dump(out, open(os.path.join(dst, "pmc_traffic.json"), "w"), indent=1)
    for k, v in sorted(kernels.items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"])[:8]:
        print(f"{k:32s} {v['hbm_bytes_per_launch'] / 1e9:9.3f} GB/launch")


if __name__ == "__main__":
    main()
