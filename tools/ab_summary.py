#!/usr/bin/env python3
"""One line per bench JSON (A/B runs): ms/step, chain tail, the largest kernels' ms per step.
usage: python tools/ab_summary.py gpurun_out/ab_*.json gpurun_out/c3_opts_*.json"""
import json
import sys

for f in sys.argv[1:]:
    d = json.load(open(f))
    k = d["roofline"].get("kernels_ms_per_step") or {}
    top = {n: round(v) for n, v in sorted(k.items(), key=lambda x: -x[1])[:10]}
    print(f"{f}: {d['ms_per_step']:.1f} ms, tail {d.get('chain_tail_ms') or 0:.1f}, {top}")
