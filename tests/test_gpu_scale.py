"""Parity at BASELINE configs[1] size (C2: 1M synthetic proteins, 4,000 families) and against the
C2-built signature DB (C4's database, all 10M fresh queries of configs[3]).

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


@pytest.mark.parametrize("passes,route_min", [(0, 0), (4, 0), (8, 2048)])
def test_c2_build_bit_exact(skm, c2, passes, route_min):
    """The whole C2 build vs the oracle, bit for bit (one pass; four key-range passes; eight with the
    k-mers of >= 2048 occurrences routed into the first four)."""
    r, o, l, f, i = c2["inputs"]
    b = skm.SignatureBuilder(len(c2["funcs"]))
    if passes:
        b.set_option("key_range_passes", passes)
        b.set_option("route_heavy_min", route_min)
    b.add_batch(r, o, l, f, i)
    b.run()
    c = b.counters()
    jobs = b.debug_jobs(8)
    got = b.finish()
    b.close()
    # the paths this size exists to reach
    assert c["overflow_subbuckets"] > 100 and c["overflow_elements"] > 10_000_000
    assert c["big_groups"] > 10_000
    # wave-pair chains of >= 2^14 samples (in situ or giant with one pass; stashed with passes --
    # with routing the last pass, whose jobs debug_jobs lists, holds no heavy k-mer)
    assert max(max(jobs), c["giant_max"]) >= 16384 or c["long_samples"] >= 16384, (jobs, c)
    if route_min:
        assert c["routed"] > 1_000_000, c
    _same(got, c2["ref"])
    c2.setdefault("kept", got)


def _pooled(n_total, first_file, n_files):
    """Files [first_file, first_file + n_files) of an n_total proteome from the bench's worker
    pool, packed (residues, seq_off, seq_len)."""
    parts = list(synth.iter_file_inputs(n_total, FAM, 4000, first_file, n_files, workers=min(16, _threads())))
    lens = np.concatenate([p[2] for p in parts])
    res = np.concatenate([p[0] for p in parts])
    off = np.zeros(len(lens), np.uint64)
    off[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    return res, off, lens


def test_c4_db_calls_bit_exact(skm, c2, tmp_path):
    """BASELINE configs[3] at full size: the calls of all 10M fresh queries (3.03 G windows, the
    bench's C4 leg: genome files 250..2749 of the C3 proteome) against the C2-built CMPH/BDZ DB
    (168.7M keys, device-peeled MPH, resident in HBM) vs process_aa_seq of the oracle on the
    same .mph/.dat image, on every host core (call_functions.tcc:259-338)."""
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
    nq = 10_000_000
    qr, qo, ql = _pooled(50_000_000, N_C2 // 4000, nq // 4000)
    assert len(ql) == nq
    db = skm.CmphKmerDb(base, device=0)
    assert db.hash_size() == len(kept.keys)
    hypo = funcs.index("hypothetical protein")
    caller = skm.FunctionCaller(db, funcs)
    off, calls = caller.process_seqs(qr, qo, ql)
    db.close()
    ob = oracle_ref.Bdz(open(base + ".mph", "rb").read())
    ooff, ocalls = oracle_ref.annotate_par(ob, open(base + ".dat", "rb").read(), qr, qo, ql, _threads(), hypo_index=hypo)
    assert int(np.where(ql >= 8, ql.astype(np.int64) - 7, 0).sum()) > 3_000_000_000
    assert len(calls) > 5_000_000
    assert np.array_equal(off, ooff)
    assert np.array_equal(calls.view(np.uint8), ocalls.view(np.uint8))


def test_c2_recall_bit_exact(skm, c2):
    """The recall pass at C2 size (kmers-build-signatures.cc:238-349): every one of the 1M training
    proteins (303M windows) called against the exact kept-k-mer DB of its own build (KeptKmerDB,
    kept_kmer_db.h:20-27: 168.7M keys, the device exact-key table) -- the calls equal process_aa_seq
    of the oracle against the sorted kept set, on every host core."""
    kept = c2.get("kept")
    if kept is None:
        r, o, l, f, i = c2["inputs"]
        b = skm.SignatureBuilder(len(c2["funcs"]))
        b.add_batch(r, o, l, f, i)
        kept = b.finish()
        b.close()
    r, o, l, _, _ = c2["inputs"]
    funcs = c2["funcs"]
    hypo = funcs.index("hypothetical protein")
    db = skm.KeptKmerDb(kept.keys, kept.data, device=0)
    caller = skm.FunctionCaller(db, funcs)
    off, calls = caller.process_seqs(r, o, l)
    db.close()
    ooff, ocalls = oracle_ref.annotate_exact_par(kept.keys, kept.data, r, o, l, _threads(), hypo_index=hypo)
    assert len(calls) > 500_000
    assert np.array_equal(off, ooff)
    assert np.array_equal(calls.view(np.uint8), ocalls.view(np.uint8))
