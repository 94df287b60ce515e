#!/usr/bin/env python3
"""Peelability of cmph's BDZ 3-graph (c = 1.23, r = ceil(c m / 3) made odd) with uniform vertices
vs the skew of a 32-bit hash reduced mod r when 2^32 / r = 3.64 (C3: r = 1.18 G): the lowest 63.7 %
of the residues have four preimages, the rest three.  CPU only (numpy, vectorised peel rounds).

usage: python tools/bdz_skew_sim.py [m] [seeds]     (m = 3,000,000, 3 seeds)
prints, per graph, (edges left in the 2-core, peel rounds)."""
import sys

import numpy as np


def peel(m, skewed, seed):
    rng = np.random.default_rng(seed)
    r = int(np.ceil(1.23 * m / 3))
    r += r % 2 == 0

    def verts():
        if not skewed:
            return rng.integers(0, r, m)
        k4 = int(0.637 * r)
        p4 = 4 * k4 / (4 * k4 + 3 * (r - k4))
        return np.where(rng.random(m) < p4, rng.integers(0, k4, m), rng.integers(k4, r, m))

    v = np.stack([verts(), verts() + r, verts() + 2 * r], 1)
    n = 3 * r
    alive = np.ones(m, bool)
    deg = np.bincount(v.ravel(), minlength=n)
    rounds = 0
    while True:
        out = alive & (deg[v] == 1).any(1)
        if not out.any():
            break
        alive[out] = False
        deg -= np.bincount(v[out].ravel(), minlength=n)
        rounds += 1
    return int(alive.sum()), rounds


if __name__ == "__main__":
    m = int(sys.argv[1]) if len(sys.argv) > 1 else 3_000_000
    seeds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    for skewed in (False, True):
        print("skewed" if skewed else "uniform", [peel(m, skewed, s) for s in range(seeds)], flush=True)
