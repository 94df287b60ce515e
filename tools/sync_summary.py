#!/usr/bin/env python3
"""Fold a tools/sync_count.sh run (gpurun_out/syncs/r1, r3: HIP runtime API statistics of the C2
probe build with 1 and 3 runs) into profiles/r02_hip_api_per_step.json: the calls one build step
adds, (calls(3 runs) - calls(1 run)) / 2, for every HIP API function -- the host synchronisations
(hipStreamSynchronize, hipEventSynchronize, hipDeviceSynchronize, blocking hipMemcpy) among them.
usage: python tools/sync_summary.py [gpurun_out/syncs]
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SYNC = ("hipStreamSynchronize", "hipEventSynchronize", "hipDeviceSynchronize", "hipMemcpy", "hipMemcpyDtoH",
        "hipMemcpyHtoD", "hipMalloc", "hipFree", "hipHostMalloc", "hipHostFree")


def calls(d):
    f = glob.glob(os.path.join(d, "**", "*hip_api_stats.csv"), recursive=True)
    assert f, f"no hip_api_stats.csv under {d}"
    out = {}
    for row in csv.DictReader(open(f[0])):
        out[row["Name"]] = int(row["Calls"])
    return out


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "syncs")
    c1, c3 = calls(os.path.join(src, "r1")), calls(os.path.join(src, "r3"))
    per = {k: (c3.get(k, 0) - c1.get(k, 0)) / 2 for k in sorted(set(c1) | set(c3))}
    per = {k: v for k, v in per.items() if v}
    out = {"round": "r02", "workload": "C2 probe build (tools/pmc_probe.py: 1,000,000 proteins, one pass)",
           "method": "rocprofv3 --hip-runtime-trace --stats, 3 runs minus 1 run, halved (tools/sync_count.sh)",
           "per_step": per,
           "host_syncs_per_step": {k: per.get(k, 0) for k in SYNC if per.get(k, 0)}}
    json.dump(out, open(os.path.join(ROOT, "profiles", "r02_hip_api_per_step.json"), "w"), indent=1)
    print(json.dumps(out["host_syncs_per_step"]))
    print({k: v for k, v in sorted(per.items(), key=lambda kv: -kv[1])[:12]})


if __name__ == "__main__":
    main()
