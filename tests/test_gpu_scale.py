"""Parity at BASELINE configs[1] size (C2: 1M synthetic proteins, 4,000 families) and against the
C2-built signature DB (C4's database, 1M fresh queries).

At this size the heaviest k-mers have ~2*10^4 occurrences: the build reaches the overflow path
(sub-buckets beyond LDS, global bitonic sort), the in-situ wave-pair P^2 chains of >= 16,384
samples (k_chain_long) and k_big_groups, none of which the small parity cases exercise at these
depths.  The oracle (oracle/skm_oracle.cpp) runs on all host cores: oracle_build_mt is the
--n-threads 1 restatement sharded by key hash (tests/test_oracle_kat.py checks it equals the
single-thread oracle), annotate_par runs the single-thread process_aa_seq restatement over
sequence ranges.  The generator is the bench's (seed 20241115)."""
import os

import numpy as np
import pytest

import oracle_ref
from signature_kmers_amd import synth

pytestmark = pytest.mark.gpu

N_C2, FAM = 1_000_000, 4000


def _threads():
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            return max(1, min(len(os.sched_getaffinity(0)), int(q) // int(p)))
    except (OSError, ValueError):
        pass
    return len(os.sched_getaffinity(0))


@pytest.fixture(scope="module")
def c2(skm, gpu):
    p = synth.generate_arrays(N_C2, FAM, per_file=4000)
    r, o, l, f, i, funcs = synth.build_inputs(p)
    ref = oracle_ref.build_mt(r, o, l, f, i, len(funcs), _threads(), sort=True)
    return dict(inputs=(r, o, l, f, i), funcs=funcs, ref=ref)


def _same(got, ref):
    assert len(got.keys) == len(ref["keys"])
    assert np.array_equal(got.keys, ref["keys"])
    assert np.array_equal(got.data.view(np.uint8), ref["data"].view(np.uint8))
    assert np.array_equal(got.distinct_functions, ref["distinct_functions"])
    assert np.array_equal(got.seqs_with_func, ref["seqs_with_func"])
    assert got.n_seqs_with_signature == ref["n_seqs_with_signature"]
    assert got.distinct_signatures == ref["distinct_signatures"]


@pytest.mark.parametrize("passes", [0, 4])
def test_c2_build_bit_exact(skm, c2, passes):
    """The whole C2 build vs the oracle, bit for bit (one pass, and four key-range passes)."""
    r, o, l, f, i = c2["inputs"]
    b = skm.SignatureBuilder(len(c2["funcs"]))
    if passes:
        b.set_option("key_range_passes", passes)
    b.add_batch(r, o, l, f, i)
    b.run()
    c = b.counters()
    jobs = b.debug_jobs(8)
    got = b.finish()
    b.close()
    # the paths this size exists to reach
    assert c["overflow_subbuckets"] > 100 and c["overflow_elements"] > 10_000_000
    assert c["big_groups"] > 10_000
    assert max(max(jobs), c["giant_max"]) >= 16384, (jobs, c)  # wave-pair chains (in situ or giant)
    _same(got, c2["ref"])
    c2.setdefault("kept", got)


def test_c4_db_calls_bit_exact(skm, c2, tmp_path):
    """Calls of 1M fresh queries against the C2-built CMPH/BDZ DB (168.7M keys, device-peeled
    MPH, resident in HBM) vs process_aa_seq of the oracle on the same .mph/.dat image."""
    kept = c2.get("kept")
    if kept is None:
        r, o, l, f, i = c2["inputs"]
        b = skm.SignatureBuilder(len(c2["funcs"]))
        b.add_batch(r, o, l, f, i)
        kept = b.finish()
        b.close()
    funcs = c2["funcs"]
    base = str(tmp_path / "kmer_data")
    skm.mph_build(kept.keys, kept.data, base + ".mph", base + ".dat", seed=1, device=0)
    nq = 1_000_000
    q = synth.generate_arrays(N_C2 + nq, FAM, per_file=4000, first_file=N_C2 // 4000, n_files=nq // 4000)
    assert len(q.seq_len) == nq
    db = skm.CmphKmerDb(base, device=0)
    assert db.hash_size() == len(kept.keys)
    hypo = funcs.index("hypothetical protein")
    caller = skm.FunctionCaller(db, funcs)
    off, calls = caller.process_seqs(q.residues, q.seq_off, q.seq_len)
    db.close()
    ob = oracle_ref.Bdz(open(base + ".mph", "rb").read())
    ooff, ocalls = oracle_ref.annotate_par(ob, open(base + ".dat", "rb").read(), q.residues, q.seq_off, q.seq_len,
                                           _threads(), hypo_index=hypo)
    assert len(calls) > 500_000
    assert np.array_equal(off, ooff)
    assert np.array_equal(calls.view(np.uint8), ocalls.view(np.uint8))
