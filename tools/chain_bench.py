"""Chain kernel latency: ns per sample of one chain (and of 64 chains) per chain code."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import signature_kmers_amd as skm  # noqa: E402

for n in (4000, 16000, 64000):
    for mode, name in ((1, "per-lane"), (2, "wave-pair"), (3, "p2-wave"), (4, "var-wave"), (5, "p2v-wave")):
        for nj in (1, 16):
            ms = skm.debug_chain_bench(n, nj, mode)
            print(f"n={n:6d} jobs={nj:3d} {name:9s}: {ms:8.3f} ms  {1e6 * ms / n:7.1f} ns/sample", flush=True)
