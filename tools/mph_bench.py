#!/usr/bin/env python3
"""Time BDZ construction (skm_mph_build host vs skm_mph_build_device) on random distinct keys."""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import signature_kmers_amd as skm  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, nargs="+", default=[20_000_000, 168_000_000])
ap.add_argument("--host-max", type=int, default=20_000_000)
ap.add_argument("--out", default="/tmp")
a = ap.parse_args()
for n in a.n:
    rng = np.random.default_rng(n)
    keys = np.unique(rng.integers(1, 2**63, size=int(n * 1.01), dtype=np.uint64))[:n]
    rng.shuffle(keys)
    data = np.zeros(len(keys), skm.STORED_DTYPE)
    t = time.time()
    skm.mph_build(keys, data, f"{a.out}/d.mph", f"{a.out}/d.dat", seed=1, device=0)
    td = time.time() - t
    th = None
    if n <= a.host_max:
        t = time.time()
        skm.mph_build(keys, data, f"{a.out}/h.mph", f"{a.out}/h.dat", seed=1)
        th = time.time() - t
    print(f"n={len(keys)} device {td:.2f} s" + (f", host {th:.2f} s" if th else ""), flush=True)
    st = skm.mph_build_device(keys, data, f"{a.out}/e.mph", f"{a.out}/e.dat", seed=1, device=0, verify=False)
    print("  skm_mph_build_device_ex phases (s):", {k: round(v, 3) if isinstance(v, float) else v for k, v in st.items()},
          flush=True)
