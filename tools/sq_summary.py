#!/usr/bin/env python3
"""Fold a tools/pmc_sq.sh run (gpurun_out/pmc_sq/p1, p2: SQ counters of the C2 probe build,
tools/pmc_probe.py, two runs; SKM_PROBE_ANNOT=1 adds the annotate path) into profiles/R_sq_counters.json
(round tag R, default r04): per kernel the summed counters
and the ratios that say what bounds it --
  wait_frac      SQ_WAIT_ANY / SQ_WAVE_CYCLES        share of wave time spent waiting (memory/LDS/barrier)
  active_frac    SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES share of wave time issuing
  lds_conflict   SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS  bank-conflict cycles per LDS-issue cycle
  valu_per_vmem  SQ_INSTS_VALU / SQ_INSTS_VMEM
usage: python tools/sq_summary.py [gpurun_out/pmc_sq] [round] [workload text] [output name]
"""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "pmc_sq")
    rnd = sys.argv[2] if len(sys.argv) > 2 else "r04"
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    launches = collections.defaultdict(set)
    for p in sorted(os.listdir(src)):
        f = os.path.join(src, p, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"].split("(")[0].replace("void ", "").replace("skm::", "")
            if not k:
                continue
            acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
            launches[(k, p)].add(row["Dispatch_Id"])
    wl = sys.argv[3] if len(sys.argv) > 3 else ("C2 probe build (tools/pmc_probe.py: 1,000,000 proteins, 2 runs) + "
                                                 "annotate of 1,000,000 fresh queries against its DB (2 runs)")
    name = sys.argv[4] if len(sys.argv) > 4 else f"{rnd}_sq_counters.json"
    out = {"round": rnd, "workload": wl,
           "script": "tools/pmc_sq.sh", "kernels": {}}
    for k, c in acc.items():
        wc = c.get("SQ_WAVE_CYCLES", 0.0)
        r = {"counters": dict(sorted(c.items()))}
        if wc:
            r["wait_frac"] = c.get("SQ_WAIT_ANY", 0.0) / wc
            r["active_frac"] = c.get("SQ_ACTIVE_INST_ANY", 0.0) / wc
        if c.get("SQ_ACTIVE_INST_LDS"):
            r["lds_conflict"] = c.get("SQ_LDS_BANK_CONFLICT", 0.0) / c["SQ_ACTIVE_INST_LDS"]
        if c.get("SQ_INSTS_VMEM"):
            r["valu_per_vmem"] = c.get("SQ_INSTS_VALU", 0.0) / c["SQ_INSTS_VMEM"]
        out["kernels"][k] = r
    json.dump(out, open(os.path.join(ROOT, "profiles", name), "w"), indent=1)
    rank = sorted(out["kernels"].items(), key=lambda kv: -kv[1]["counters"].get("SQ_WAVE_CYCLES", 0))
    for k, r in rank[:10]:
        print(f"{k:24s} wave_cycles {r['counters'].get('SQ_WAVE_CYCLES', 0):.3g} "
              f"wait {r.get('wait_frac', 0):.2f} active {r.get('active_frac', 0):.2f} "
              f"lds_conflict {r.get('lds_conflict', 0):.2f} valu/vmem {r.get('valu_per_vmem', 0):.1f}")


if __name__ == "__main__":
    main()
