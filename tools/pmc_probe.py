"""Small workload for counter passes: one C2 build, two runs; with SKM_PROBE_ANNOT=1 also the
annotate path (the build's kept set as a CMPH/BDZ DB, 1M fresh queries of the same families,
two runs: k_lookup, k_calls_scan, k_seg_process)."""
import os, sys, tempfile
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import signature_kmers_amd as skm
from signature_kmers_amd import synth
n = int(os.environ.get("SKM_PROBE_SEQS", "1000000"))
p = synth.generate_arrays(n, 4000, per_file=4000)
r, o, l, f, i, funcs = synth.build_inputs(p)
b = skm.SignatureBuilder(len(funcs))
b.add_batch(r, o, l, f, i)
b.prepare()
for _ in range(int(os.environ.get('SKM_PROBE_RUNS', '2'))):
    b.run()
print(b.timings())
if os.environ.get("SKM_PROBE_ANNOT") == "1":
    kept = b.finish()
    b.close()
    q = synth.generate_arrays(2 * n, 4000, per_file=4000, first_file=n // 4000, n_files=max(1, n // 4000))
    with tempfile.TemporaryDirectory(dir="/tmp") as d:
        base = os.path.join(d, "kmer_data")
        skm.mph_build(kept.keys, kept.data, base + ".mph", base + ".dat", seed=1, device=0)
        db = skm.CmphKmerDb(base, device=0)
    qb = skm.QueryBatch(db, q.residues, q.seq_off, q.seq_len)
    hypo = funcs.index("hypothetical protein")
    for _ in range(int(os.environ.get('SKM_PROBE_RUNS', '2'))):
        qb.run(hypo)
    print(qb.timings())
    qb.close()
    db.close()
