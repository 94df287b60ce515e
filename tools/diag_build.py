"""Diagnostics for the device build: phase timings, counters and k_bucket_process phase stamps."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import signature_kmers_amd as skm  # noqa: E402
from signature_kmers_amd import synth  # noqa: E402

STAMP_NAMES = {0: "l2_count", 1: "l2_scatter", 9: "l2_setup", 2: "sub_load", 3: "sub_hash", 4: "sub_classify",
               5: "sub_scatter", 6: "sub_class_sort", 11: "sub_seg_groups", 7: "sub_big_groups", 8: "sub_emit",
               10: "sub_loop_tail"}

ap = argparse.ArgumentParser()
ap.add_argument("--seqs", type=int, default=1_000_000)
ap.add_argument("--families", type=int, default=4000)
ap.add_argument("--steps", type=int, default=2)
a = ap.parse_args()
t = time.time()
p = synth.generate_arrays(a.seqs, a.families)
r, o, l, f, i, funcs = synth.build_inputs(p)
print("gen", round(time.time() - t, 1), "s", flush=True)
b = skm.SignatureBuilder(len(funcs))
b.add_batch(r, o, l, f, i)
b.prepare()
b.run()
print("timings", json.dumps(b.timings()))
b.debug_stamps(True)
b.run()
st = b.debug_stamps(False)
tot = sum(st[:16])
print("stamps (cycles summed over workgroups):")
for k in sorted(STAMP_NAMES):  # noqa
    print(f"  {STAMP_NAMES[k]:>20s} {st[k]:>16d} {100.0 * st[k] / max(tot, 1):6.1f}%")
for q, nm in enumerate(["65-128", "129-256", "257-512", "513-2048"]):
    ng = st[20 + q]
    print(f"  big groups {nm:>9s}: {ng:>9d} groups, {st[16 + q] / max(ng, 1):10.0f} cycles/group (wave), "
          f"{100.0 * st[16 + q] / max(tot, 1):5.1f}% of stamped WG cycles")
print("timings(stamped)", json.dumps(b.timings()))
print("counters", json.dumps(b.counters()))
print("longest jobs", b.debug_jobs(16))
for n, nj in [(1000, 1), (1000, 64), (1000, 4096), (16000, 1), (16000, 64), (100, 100000), (10, 1000000)]:
    print("chain bench n=%d jobs=%d: %.3f ms" % (n, nj, skm.debug_chain_bench(n, nj)))
for _ in range(a.steps):
    b.run()
    print("timings", json.dumps(b.timings()))
