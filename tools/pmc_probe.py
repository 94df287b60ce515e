"""Small workload for counter passes: one C2 build, two runs."""
import os, sys
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
