#!/usr/bin/env python3
"""Fold a tools/gpu_profile.sh run (gpurun_out/) into profiles/ (round tag R, default r05):

profiles/R_kernel_stats_{c3,c2,legs}.csv     rocprofv3 --kernel-trace --stats summaries
profiles/R_pmc_traffic.json                  per kernel and workload: counter KiB per build run (c3,
                                             c2: one run each) or per launch (legs), and HBM bytes
                                             corrected by the calibrated factor of the kernel's access
                                             shape (profiles/r02_fetch_calib.json: coalesced streaming
                                             reads are counted at 1/2 (x2), random 8-byte gathers at one
                                             64-byte request each (x1)); stamped with src_sha16, the
                                             hash of the device sources it was taken on -- bench.py
                                             uses a kernel's traffic only for the same sources
usage: python tools/pmc_summary.py [gpurun_out] [round]
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GATHER_KERNELS = {"k_lookup<0>", "k_lookup<1>", "k_md_hits", "k_mph_place", "k_mph_assign"}


def per_kernel(path, counter):
    acc = collections.defaultdict(list)
    for row in csv.DictReader(open(path)):
        if row["Counter_Name"] != counter:
            continue
        name = row["Kernel_Name"].split("(")[0].replace("void ", "").replace("skm::", "")
        for base in ("k_extract_stage_pos", "k_pass_emit", "k_partition"):  # variants share one row (bench.py)
            if name.startswith(base + "<"):
                name = base
        acc[name].append(float(row["Counter_Value"]))
    return acc


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out")
    rnd = sys.argv[2] if len(sys.argv) > 2 else "r05"
    dst = os.path.join(ROOT, "profiles")
    for w in ("c3", "c2", "legs"):
        p = os.path.join(src, f"prof_{w}", "run_kernel_stats.csv")
        if os.path.exists(p):
            shutil.copy(p, os.path.join(dst, f"{rnd}_kernel_stats_{w}.csv"))
    sha = open(os.path.join(src, "src_sha16.txt")).read().strip()
    out = {"round": rnd, "src_sha16": sha,
           "formula": "(f * FETCH_SIZE + WRITE_SIZE) * 1024; f = 2 for streaming kernels, 1 for gather kernels "
                      "(profiles/r02_fetch_calib.json)",
           "gather_kernels": sorted(GATHER_KERNELS),
           "workloads": {"c3": {"seqs": 50000000, "unit": "per build run (16 key-range passes)"},
                         "c2": {"seqs": 1000000, "unit": "per build run"},
                         "legs": {"queries": 10000000, "matrix_seqs": 100000, "recall_proteins": 1000000,
                                  "unit": "per launch"}},
           "kernels": {}}
    for w in ("c3", "c2", "legs"):
        fp = os.path.join(src, f"pmc_{w}_fetch", "run_counter_collection.csv")
        wp = os.path.join(src, f"pmc_{w}_write", "run_counter_collection.csv")
        if not (os.path.exists(fp) and os.path.exists(wp)):
            continue
        f, wr = per_kernel(fp, "FETCH_SIZE"), per_kernel(wp, "WRITE_SIZE")
        for k in sorted(set(f) | set(wr)):
            fv, wv = f.get(k, [0.0]), wr.get(k, [0.0])
            if w == "legs":
                fk, wk = sum(fv) / len(fv), sum(wv) / len(wv)
            else:
                fk, wk = sum(fv), sum(wv)
            fac = 1.0 if k in GATHER_KERNELS else 2.0
            out["kernels"].setdefault(k, {})[w] = {"FETCH_SIZE_KiB": fk, "WRITE_SIZE_KiB": wk, "launches": len(fv),
                                                   "fetch_factor": fac, "hbm_bytes": (fac * fk + wk) * 1024}
    json.dump(out, open(os.path.join(dst, f"{rnd}_pmc_traffic.json"), "w"), indent=1)
    tot = collections.Counter()
    for k, v in out["kernels"].items():
        for w, x in v.items():
            tot[w] += x["hbm_bytes"]
    print("total HBM bytes per run/launch-set:", {w: round(b / 1e9, 1) for w, b in tot.items()})
    for k in sorted(out["kernels"], key=lambda k: -out["kernels"][k].get("c3", {}).get("hbm_bytes", 0))[:14]:
        print(k, {w: round(v["hbm_bytes"] / 1e9, 2) for w, v in out["kernels"][k].items()})


if __name__ == "__main__":
    main()
