"""Known-answer tests pinning the CPU oracle (oracle/skm_oracle.cpp) to the reference semantics.

The reference ships no tests or golden vectors, so parity is unpinned by the
reference itself.  These KATs are derived by hand from the reference source (file:line cited per
test) and SURVEY.md Appendix A; a second, independently written Python restatement (pyref.py)
cross-checks the oracle on randomized small inputs.
"""
import numpy as np
import pytest

import oracle_ref
import pyref

KEY = int.from_bytes(b"MKVLAAGW", "little")


def pack(seqs, funcs, ids=None):
    lens = np.array([len(s) for s in seqs], np.uint32)
    off = np.zeros(len(seqs), np.uint64)
    if len(seqs) > 1:
        off[1:] = np.cumsum(lens[:-1].astype(np.uint64))
    res = np.frombuffer(b"".join(seqs), np.uint8) if sum(map(len, seqs)) else np.zeros(0, np.uint8)
    ids = np.arange(len(seqs), dtype=np.uint32) if ids is None else np.asarray(ids, np.uint32)
    return res, off, lens, np.asarray(funcs, np.uint16), ids


def obuild(seqs, funcs, nf, ids=None):
    return oracle_ref.build(*pack(seqs, funcs, ids), nf)


def as_dict(ref):
    return {int(k): tuple(int(x) for x in d) for k, d in zip(ref["keys"], ref["data"])}


def test_two_windows_singletons():
    # signature_build.tcc:162-178 windows i in [0, len-8]; offset = len - i; singletons always pass
    r = as_dict(obuild([b"ACDEFGHIK"], [0], 1))
    k0 = int.from_bytes(b"ACDEFGHI", "little")
    k1 = int.from_bytes(b"CDEFGHIK", "little")
    # (avg_from_end, function_index, mean, median, var); P^2 median of n <= 2 samples is 0
    assert r == {k0: (9, 0, 9, 0, 0), k1: (8, 0, 9, 0, 0)}


@pytest.mark.parametrize("funcs,kept", [([0, 0, 0, 0, 1], True),     # 4 >= 5*0.8
                                        ([0, 0, 0, 1], False),       # 3 < 3.2
                                        ([1, 0], False),             # tie -> lowest index, 1 < 1.6
                                        ([2] * 8 + [0, 1], True),    # 8 >= 8.0
                                        ([2] * 7 + [0, 1, 0], False)])
def test_cut(funcs, kept):
    # signature_build.tcc:250-257: reject if (float)best < float(count) * 0.8f
    seqs = [b"MKVLAAGW"] * len(funcs)
    ref = obuild(seqs, funcs, 3)
    assert (KEY in as_dict(ref)) == kept
    assert ref["distinct_signatures"] == int(kept)
    if kept:
        best = max(set(funcs), key=funcs.count)
        assert as_dict(ref)[KEY][1] == best
        assert ref["distinct_functions"][best] == 1
        assert ref["n_seqs_with_signature"] == len(funcs)   # every occurrence's seq_id (:266-273)


def test_lifo_visit_order_median():
    # TBB 2020 multimap visits duplicates in reverse insertion order: the P^2 median
    # of 3 samples is the third visited = the FIRST inserted.
    seqs = [b"MKVLAAGW" + b"B" * 2, b"MKVLAAGW" + b"B" * 12, b"MKVLAAGW" + b"B" * 22]
    r = as_dict(obuild(seqs, [0, 0, 0], 1))
    # avg_from_end = sorted(10,20,30)[1]; mean 20; median 10 (LIFO); var = 25*2/3 + 100/2
    assert r == {KEY: (20, 0, 20, 10, 66)}


def test_u16_sum_wrap_and_var_overflow():
    # accumulator sum is unsigned short: 5 * 65535 wraps; the variance passes 2^31 and
    # (unsigned short)(double) follows cvttsd2si (integer-indefinite -> 0)
    seq = b"MKVLAAGW" + b"B" * (65535 - 8)
    r = as_dict(obuild([seq] * 5, [0] * 5, 1))
    assert r == {KEY: (65535, 0, 13106, 65535, 0)}


def test_u16_offset_and_mean_wrap_two():
    seqs = [b"MKVLAAGW" + b"B" * (40000 - 8), b"MKVLAAGW" + b"B" * (40001 - 8)]
    r = as_dict(obuild(seqs, [0, 0], 1))
    # sum = 80001 mod 65536 = 14465 -> mean 7232; var = 32767.5^2 -> int32 1073709056 -> u16 32768
    assert r == {KEY: (40001, 0, 7232, 0, 32768)}


def test_stats_only_over_best_function():
    # signature_build.tcc:262-275: lengths of best-function occurrences only; offsets over all
    seqs = [b"MKVLAAGW" + b"B" * k for k in (0, 10, 20, 30, 40)]
    r = as_dict(obuild(seqs, [0, 0, 0, 0, 1], 2))
    # best 0: lengths visited 38, 28, 18, 8 -> mean 23, median = 3rd visited = 18
    # var: n2 sum 66 m33 x28 -> 25; n3 sum 84 m28 x18 -> 25*2/3+100/2; n4 sum 92 m23 x8 -> *3/4 + 225/3
    v = 25.0
    v = v * 2 / 3 + 100 / 2
    v = v * 3 / 4 + 225 / 3
    # avg_from_end over ALL five offsets 8,18,28,38,48 -> 28
    assert r == {KEY: (28, 0, 23, 18, int(v))}


def test_window_validity_and_case():
    # ok_prot_ (signature_build.h:102-103): 20 amino acids, both cases; B/Z/U/X/* invalid
    seqs = [b"acdefghiB", b"ACDEFGHX", b"ACDEZGHIK", b"short", b""]
    ref = obuild(seqs, [0, 0, 0, 0, 0], 1)
    assert as_dict(ref) == {int.from_bytes(b"acdefghi", "little"): (9, 0, 9, 0, 0)}
    assert list(ref["seqs_with_func"]) == [5]      # counted before the length check (:160-162)
    assert oracle_ref.count_windows(np.array([9, 8, 9, 5, 0], np.uint32), np.zeros(5, np.uint16)) == 2 + 1 + 2


def test_skipped_function_and_colliding_ids():
    # seq_func == 0xFFFF: sequence skipped entirely (signature_build.tcc:133-158)
    seqs = [b"MKVLAAGW", b"MKVLAAGW", b"MKVLAAGW", b"MKVLAAGWA"]
    ref = obuild(seqs, [0, 0xFFFF, 0, 0], 1, ids=[7, 8, 7, 9])
    assert list(ref["seqs_with_func"]) == [3]
    assert as_dict(ref)[KEY] == (8, 0, 8, 8, 0)
    # seq ids 7 (twice, colliding) and 9 -> 2 distinct
    assert ref["n_seqs_with_signature"] == 2


def test_empty():
    ref = obuild([], [], 4)
    assert len(ref["keys"]) == 0 and ref["n_seqs_with_signature"] == 0
    assert list(ref["seqs_with_func"]) == [0, 0, 0, 0]


def test_call_side_window_iterator():
    # for_each_kmer (kmer_data.h:76-102): only 'X' / '*' are ambiguous; off-by-one skips the window
    # that ends right before the ambiguous char
    k = int.from_bytes(b"ACDEFGHI", "little")
    assert pyref.call_windows(b"ACDEFGHI") == [(0, k)]
    assert pyref.call_windows(b"ACDEFGHI*") == []
    assert pyref.call_windows(b"ACDEFGHIK*") == [(0, k)]
    assert pyref.call_windows(b"XACDEFGHI") == [(1, k)]
    assert [o for o, _ in pyref.call_windows(b"acdefghiBZU")] == [0, 1, 2, 3]
    assert pyref.call_windows(b"ACDEFGH") == []


def _rand_seqs(rng, n, alphabet, lmin, lmax, motif_p):
    motifs = [bytes(rng.choice(alphabet, 8)) for _ in range(6)]
    seqs = []
    for _ in range(n):
        L = int(rng.integers(lmin, lmax))
        s = bytearray(rng.choice(alphabet, L))
        for _ in range(int(rng.integers(0, 4))):
            if L >= 8 and rng.random() < motif_p:
                p = int(rng.integers(0, L - 7))
                s[p:p + 8] = motifs[int(rng.integers(0, len(motifs)))]
        seqs.append(bytes(s))
    return seqs


@pytest.mark.parametrize("seed", range(12))
def test_oracle_matches_python_restatement(seed):
    rng = np.random.default_rng(1000 + seed)
    alpha = np.frombuffer(b"ACDEFGHIKLMNPQRSTVWYacdX*B", np.uint8) if seed % 3 == 0 \
        else np.frombuffer(b"ACDEG", np.uint8)  # tiny alphabet -> heavy groups, long P^2 chains
    nf = int(rng.integers(1, 5))
    seqs = _rand_seqs(rng, int(rng.integers(1, 60)), alpha, 0, 90, 0.7)
    funcs = [int(x) if rng.random() > 0.1 else 0xFFFF for x in rng.integers(0, nf, len(seqs))]
    ids = [int(x) for x in rng.integers(0, 40, len(seqs))]
    exp, dist, swf, nsig = pyref.build_py(seqs, funcs, ids, nf)
    ref = obuild(seqs, funcs, nf, ids)
    assert as_dict(ref) == exp
    assert list(ref["distinct_functions"]) == dist
    assert list(ref["seqs_with_func"]) == swf
    assert ref["n_seqs_with_signature"] == nsig
    assert ref["distinct_signatures"] == len(exp)
    assert np.all(np.diff(ref["keys"].astype(np.uint64)) > 0)  # strictly ascending


@pytest.mark.parametrize("threads", [1, 3, 8])
def test_multithreaded_port_equals_single_thread(threads):
    """oracle_build_mt (bench.py's all-core CPU baseline) == oracle_build, incl. colliding ids."""
    from signature_kmers_amd import synth
    p = synth.generate_arrays(3000, 30, per_file=300, extras=True)
    r, o, l, f, i, funcs = synth.build_inputs(p)
    i = (i % 700).astype(np.uint32)  # colliding seq_ids
    a = oracle_ref.build(r, o, l, f, i, len(funcs))
    b = oracle_ref.build_mt(r, o, l, f, i, len(funcs), threads)
    assert np.array_equal(a["keys"], b["keys"])
    assert np.array_equal(a["data"].view(np.uint8), b["data"].view(np.uint8))
    for k in ("distinct_functions", "seqs_with_func"):
        assert np.array_equal(a[k], b[k])
    assert a["n_seqs_with_signature"] == b["n_seqs_with_signature"]
    assert a["distinct_signatures"] == b["distinct_signatures"]
