#!/usr/bin/env python3
"""Fold a tools/gpu_profile_r02.sh run (gpurun_out/) into profiles/:

profiles/r02_kernel_stats_{c3,c2,legs}.csv   rocprofv3 --kernel-trace --stats summaries
profiles/r02_fetch_calib.json                FETCH_SIZE / WRITE_SIZE of bin/fetch_calib's kernels
                                             against their known byte counts
profiles/r02_pmc_traffic.json                per kernel and workload: counter KiB per build run (c3,
                                             c2: one run each) or per launch (legs), and HBM bytes
                                             corrected by the calibrated factor of the kernel's
                                             access shape: coalesced streaming reads are counted at
                                             1/2 (x2), random 8-byte gathers at one 64-byte request
                                             each, which is what the DRAM moves (x1)
usage: python tools/pmc_summary_r02.py [gpurun_out]
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# kernels whose reads are dominated by independent random gathers (calibrated at 64 B / request)
GATHER_KERNELS = {"k_lookup<0>", "k_lookup<1>", "k_md_hits", "k_mph_place", "k_mph_assign"}


def per_kernel(path, counter):
    acc = collections.defaultdict(list)
    for row in csv.DictReader(open(path)):
        if row["Counter_Name"] != counter:
            continue
        name = row["Kernel_Name"].split("(")[0].replace("void ", "").replace("skm::", "")
        acc[name].append(float(row["Counter_Value"]))
    return acc


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out")
    dst = os.path.join(ROOT, "profiles")
    for w in ("c3", "c2", "legs"):
        shutil.copy(os.path.join(src, f"prof_{w}", "run_kernel_stats.csv"), os.path.join(dst, f"r02_kernel_stats_{w}.csv"))
    known = json.load(open(os.path.join(src, "calib.json")))
    cf = per_kernel(os.path.join(src, "pmc_calib_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    cw = per_kernel(os.path.join(src, "pmc_calib_write", "run_counter_collection.csv"), "WRITE_SIZE")
    calib = {k: {"bytes": b, "FETCH_SIZE_bytes": 1024 * sum(cf.get(k, [0])), "WRITE_SIZE_bytes": 1024 * sum(cw.get(k, [0])),
                 "fetch_ratio": 1024 * sum(cf.get(k, [0])) / b, "write_ratio": 1024 * sum(cw.get(k, [0])) / b}
             for k, b in known.items()}
    json.dump({"round": "r02", "probe": "tools/probes/fetch_calib.hip (4 GiB buffers, one dispatch each)",
               "kernels": calib}, open(os.path.join(dst, "r02_fetch_calib.json"), "w"), indent=1)
    out = {"round": "r02",
           "formula": "(f * FETCH_SIZE + WRITE_SIZE) * 1024; f = 2 for streaming kernels, 1 for gather kernels "
                      "(profiles/r02_fetch_calib.json)",
           "gather_kernels": sorted(GATHER_KERNELS),
           "workloads": {"c3": {"seqs": 50000000, "unit": "per build run (16 key-range passes)"},
                         "c2": {"seqs": 1000000, "unit": "per build run"},
                         "legs": {"queries": 10000000, "matrix_seqs": 100000, "unit": "per launch"}},
           "kernels": {}}
    for w in ("c3", "c2", "legs"):
        f = per_kernel(os.path.join(src, f"pmc_{w}_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
        wr = per_kernel(os.path.join(src, f"pmc_{w}_write", "run_counter_collection.csv"), "WRITE_SIZE")
        for k in sorted(set(f) | set(wr)):
            fv, wv = f.get(k, [0.0]), wr.get(k, [0.0])
            if w == "legs":
                fk, wk = sum(fv) / len(fv), sum(wv) / len(wv)
            else:
                fk, wk = sum(fv), sum(wv)
            fac = 1.0 if k in GATHER_KERNELS else 2.0
            out["kernels"].setdefault(k, {})[w] = {"FETCH_SIZE_KiB": fk, "WRITE_SIZE_KiB": wk, "launches": len(fv),
                                                   "fetch_factor": fac, "hbm_bytes": (fac * fk + wk) * 1024}
    json.dump(out, open(os.path.join(dst, "r02_pmc_traffic.json"), "w"), indent=1)
    for k in ("k_bucket_process", "k_partition", "k_extract_stage_pos", "k_split_stage", "k_lookup<0>", "k_md_rows"):
        print(k, {w: round(v["hbm_bytes"] / 1e9, 2) for w, v in out["kernels"].get(k, {}).items()})


if __name__ == "__main__":
    main()
