#!/usr/bin/env python3
"""The kept-set hand-off (skm_build_finish) at a bench size: generate the C2 (or C3) proteome as
bench.py does, build it once on the GPU, time finish() and check the result's shape (keys strictly
ascending, n == the run's kept count).  usage: python tools/finish_probe.py [--seqs N] [--slices B]"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seqs", type=int, default=1_000_000)
    ap.add_argument("--slices", type=int, default=0, help="also time finish_slice over 2^B slices")
    a = ap.parse_args()
    from signature_kmers_amd import synth
    t = time.time()
    sh = bench.gen(synth, a.seqs, 4000, 0, (a.seqs + bench.PER_FILE - 1) // bench.PER_FILE, 16)
    bench.log(f"generated {sh.n_seqs:,} proteins in {time.time() - t:.1f} s")
    import signature_kmers_amd as skm
    skm.warm_device(0)
    b = skm.SignatureBuilder(len(synth.functions(4000)), device=0)
    sh.add_to(b)
    b.prepare()
    b.run()
    b.run()
    c = b.counters()
    bench.log(f"built: kept {c['kept']:,}, {b.timings()['total']:.1f} ms device")
    res = {"seqs": a.seqs, "kept": c["kept"]}
    for rep in range(2):
        t = time.perf_counter()
        k = b.finish()
        dt = time.perf_counter() - t
        c = b.counters()
        ok = len(k.keys) == c["kept"] and bool(np.all(k.keys[1:] > k.keys[:-1]))
        res[f"finish_s_{rep}"] = dt
        res[f"handoff_{rep}"] = {x: c[x] for x in ("finish_us", "finish_wait_us", "finish_copy_us", "finish_chunks",
                                                    "finish_select_dev_us", "finish_sort_dev_us", "finish_gather_dev_us",
                                                    "finish_d2h_dev_us")}
        bench.log(f"finish {dt:.3f} s ({res[f'handoff_{rep}']}), sorted+complete: {ok}")
        assert ok
        del k
    if a.slices:
        t = time.perf_counter()
        tot = 0
        for s in range(1 << a.slices):
            k = b.finish_slice(a.slices, s)
            tot += len(k.keys)
            del k
        res["finish_slices_s"] = time.perf_counter() - t
        assert tot == c["kept"]
        bench.log(f"finish_slice x{1 << a.slices}: {res['finish_slices_s']:.3f} s")
    b.close()
    print(res, flush=True)


if __name__ == "__main__":
    main()
