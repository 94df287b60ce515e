"""C3 (50M-protein) build diagnostics on one GPU: per-phase timings, counters, the last pass's
overflow sub-bucket sizes, the longest chain jobs, and the chain kernels' per-sample latency.
Inputs come from bench.py's generator cache (python bench.py --cache-dir D --cache-only first).
    python tools/c3_diag.py --cache-dir /tmp/c3 [--option name=value ...]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import signature_kmers_amd as skm  # noqa: E402
from signature_kmers_amd import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--cache-dir", required=True)
ap.add_argument("--seqs-total", type=int, default=50_000_000)
ap.add_argument("--families", type=int, default=4000)
ap.add_argument("--steps", type=int, default=1)
ap.add_argument("--option", action="append", default=[])
ap.add_argument("--chain-bench", action="store_true")
ap.add_argument("--files", type=int, default=0, help="only the first N genome files (250 = the C2 workload)")
ap.add_argument("--runs", type=int, default=0, help="builds to run (default: steps + 1, or 6 with --files)")
ap.add_argument("--stamps", action="store_true", help="one more run with k_bucket_process phase stamps")
a = ap.parse_args()


def log(m):
    print(f"[diag] {m}", flush=True)


if a.chain_bench:
    for n in (1 << 16, 1 << 20):
        for mode, nm in ((2, "wave pair"), (3, "P2 wave"), (4, "var wave")):
            ms = skm.debug_chain_bench(n, 1, mode)
            log(f"chain n={n} {nm}: {ms:.2f} ms = {1e6 * ms / n:.1f} ns/sample")
files = (a.seqs_total + bench.PER_FILE - 1) // bench.PER_FILE
sh = bench.gen(synth, a.seqs_total, a.families, 0, files, 1, a.cache_dir)
if a.files:
    sh = bench.Shard(sh.parts[:a.files])
log(f"{sh.n_seqs:,} proteins, {sh.n_windows:,} windows")
b = skm.SignatureBuilder(len(synth.functions(a.families)))
for kv in a.option:
    k, v = kv.split("=", 1)
    b.set_option(k, int(v))
sh.add_to(b)
t = time.time()
b.prepare()
log(f"prepare {time.time() - t:.1f} s")
for s in range(a.runs or (a.steps + (1 if a.files == 0 else 5))):
    t = time.time()
    b.run()
    log(f"run {s}: {1000 * (time.time() - t):.0f} ms wall; " + json.dumps({k: round(v, 1) for k, v in b.timings().items()}))
if a.stamps:
    b.debug_stamps(True)
    b.run()
    st = b.debug_stamps(False)
    tot = sum(st[:16])
    names = {0: "l2_count", 1: "l2_scatter", 9: "l2_setup", 2: "sub_load", 3: "sub_hash", 4: "sub_classify",
             5: "sub_scatter", 6: "sub_class_sort", 11: "sub_seg_groups", 7: "sub_big_groups", 8: "sub_emit",
             10: "sub_loop_tail"}
    log("stamps (cycles summed over workgroups):")
    for k in sorted(names):
        log(f"  {names[k]:>20s} {st[k]:>16d} {100.0 * st[k] / max(tot, 1):6.1f}%")
    log("timings(stamped) " + json.dumps({k: round(v, 1) for k, v in b.timings().items()}))
c = b.counters()
log("counters " + json.dumps(c))
ov = b.debug_overflow(1 << 16)
if ov:
    import numpy as np
    v = np.array(ov, np.int64)
    log(f"last pass overflow: {len(v)} sub-buckets, {v.sum():,} elements; largest {ov[:16]}")
    for lim in (1 << 12, 1 << 14, 1 << 16, 1 << 18, 1 << 20):
        sel = v >= lim
        log(f"  >= {lim:>8d}: {int(sel.sum()):6d} sub-buckets, {int(v[sel].sum()):>12,} elements")
log(f"longest jobs (last pass) {b.debug_jobs(32)}")
b.close()
