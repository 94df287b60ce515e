"""Chain kernel throughput (k_chains, one chain per lane) at full-chip width: n samples per chain,
enough chains for ~n_total samples; prints ns per sample chip-wide and per lane."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import signature_kmers_amd as skm

for n in (4, 8, 16, 64, 200, 1000, 4000):
    nj = max(64, (64 << 20) // n)
    ms = skm.debug_chain_bench(n, nj, 1)
    print(f"n={n:5d} jobs={nj:9d} {ms:8.2f} ms  {1e6 * ms / (n * nj):7.3f} ns/sample chip-wide  "
          f"{n * nj / ms / 1e6:6.1f} G samples/s", flush=True)
