import os, sys, json
sys.path.insert(0, "/root/repo")
import signature_kmers_amd as skm
from signature_kmers_amd import synth
p = synth.generate_arrays(1000000, 4000, per_file=4000)
r, o, l, f, i, funcs = synth.build_inputs(p)
b = skm.SignatureBuilder(len(funcs))
b.add_batch(r, o, l, f, i)
b.prepare()
for e in ["0", "1", "0", "1"]:
    os.environ["SKM_EXPERIMENT"] = e
    b.run(); b.run()
    t = b.timings()
    print(e, json.dumps({k: round(v, 3) for k, v in t.items()}), flush=True)
