"""Committed golden fixtures (tests/golden/, made by tests/golden/make_golden.py).

CPU: the oracle and the host product code reproduce the fixtures.  GPU: the HIP build and
annotate paths reproduce them bit for bit.  (Parity with the reference itself is unpinned: the
reference ships no vectors)"""
import os
import sys

import numpy as np
import pytest

import oracle_ref

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
sys.path.insert(0, GOLD)
import make_golden  # noqa: E402


@pytest.fixture(scope="module")
def c1():
    g = np.load(os.path.join(GOLD, "c1_build.npz"), allow_pickle=False)
    r, o, l, f, i, funcs = make_golden.c1_inputs()
    assert make_golden.digest(r, o, l, f, i) == str(g["input_sha256"]), "synthetic C1 input drifted"
    assert list(g["functions"]) == funcs
    return g, (r, o, l, f, i, funcs)


@pytest.fixture(scope="module")
def annot():
    g = np.load(os.path.join(GOLD, "annot_small.npz"), allow_pickle=False)
    qr, qo, ql = make_golden.query_inputs()
    assert make_golden.digest(qr, qo, ql) == str(g["query_sha256"]), "synthetic query input drifted"
    return g, (qr, qo, ql)


def test_oracle_reproduces_c1(c1):
    g, (r, o, l, f, i, funcs) = c1
    ref = oracle_ref.build(r, o, l, f, i, len(funcs))
    np.testing.assert_array_equal(ref["keys"], g["keys"])
    np.testing.assert_array_equal(ref["data"].view(np.uint16).reshape(-1, 5), g["data"])
    np.testing.assert_array_equal(ref["distinct_functions"], g["distinct_functions"])
    np.testing.assert_array_equal(ref["seqs_with_func"], g["seqs_with_func"])
    assert ref["n_seqs_with_signature"] == int(g["n_seqs_with_signature"])
    assert ref["distinct_signatures"] == int(g["distinct_signatures"]) == len(g["keys"])
    assert oracle_ref.count_windows(l, f) == int(g["n_windows"])


def test_oracle_reproduces_annot(annot):
    g, (qr, qo, ql) = annot
    funcs = list(g["functions"])
    ob = oracle_ref.Bdz(g["mph"].tobytes())
    hypo = funcs.index("hypothetical protein")
    for ig, ko, kc in ((0, "call_off", "calls"), (1, "call_off_nohypo", "calls_nohypo")):
        off, calls = oracle_ref.annotate(ob, g["dat"].tobytes(), qr, qo, ql, hypo_index=hypo, ignore_hypo=ig)
        np.testing.assert_array_equal(off, g[ko])
        np.testing.assert_array_equal(calls.view(np.uint8).reshape(-1, 24), g[kc])


def test_parallel_oracle_annotate_equals_single_thread(annot):
    """annotate_par (the C2-scale GPU parity checker) is the single-thread restatement over
    sequence ranges: the same CSR calls as the golden fixture, for several thread counts."""
    g, (qr, qo, ql) = annot
    funcs = list(g["functions"])
    ob = oracle_ref.Bdz(g["mph"].tobytes())
    hypo = funcs.index("hypothetical protein")
    for t in (1, 3, 8):
        off, calls = oracle_ref.annotate_par(ob, g["dat"].tobytes(), qr, qo, ql, t, hypo_index=hypo)
        np.testing.assert_array_equal(off, g["call_off"])
        np.testing.assert_array_equal(calls.view(np.uint8).reshape(-1, 24), g["calls"])


def test_host_mph_build_reproduces_golden_image(skm, annot, tmp_path):
    g, _ = annot
    keys = g["db_keys"]
    d = np.frombuffer(g["dat"].tobytes(), skm.STORED_DTYPE)
    ob = oracle_ref.Bdz(g["mph"].tobytes())
    data = d[ob.search(keys)]     # records in key order
    base = str(tmp_path / "kmer_data")
    skm.mph_build(keys, data, base + ".mph", base + ".dat", seed=7)
    assert open(base + ".mph", "rb").read() == g["mph"].tobytes()
    assert open(base + ".dat", "rb").read() == g["dat"].tobytes()


def test_host_find_best_call_reproduces_golden(skm, annot):
    g, (qr, qo, ql) = annot
    funcs = list(g["functions"])
    calls = g["calls"].reshape(-1).view(oracle_ref.CALL_DTYPE)
    off = g["call_off"]
    for s in range(len(ql)):
        fi, fn, score, _ = skm.find_best_call(calls[off[s]:off[s + 1]], funcs)
        assert fi == g["best_fi"][s] and fn == g["best_func"][s] and np.float32(score) == g["best_score"][s], s


@pytest.mark.gpu
def test_gpu_build_reproduces_c1(skm, gpu, c1):
    g, (r, o, l, f, i, funcs) = c1
    b = skm.SignatureBuilder(len(funcs), device=gpu)
    b.add_batch(r, o, l, f, i)
    got = b.finish()
    b.close()
    np.testing.assert_array_equal(got.keys, g["keys"])
    np.testing.assert_array_equal(got.data.view(np.uint16).reshape(-1, 5), g["data"])
    np.testing.assert_array_equal(got.distinct_functions, g["distinct_functions"])
    np.testing.assert_array_equal(got.seqs_with_func, g["seqs_with_func"])
    assert got.n_seqs_with_signature == int(g["n_seqs_with_signature"])


@pytest.mark.gpu
def test_gpu_annotate_reproduces_golden(skm, gpu, annot):
    g, (qr, qo, ql) = annot
    funcs = list(g["functions"])
    db = skm.CmphKmerDb(mph=g["mph"].tobytes(), dat=g["dat"].tobytes(), device=gpu)
    caller = skm.FunctionCaller(db, funcs)
    for ig, ko, kc in ((False, "call_off", "calls"), (True, "call_off_nohypo", "calls_nohypo")):
        caller.ignore_hypothetical(ig)
        off, calls = caller.process_seqs(qr, qo, ql)
        np.testing.assert_array_equal(off, g[ko])
        np.testing.assert_array_equal(calls.view(np.uint8).reshape(-1, 24), g[kc])
    db.close()


@pytest.fixture(scope="module")
def matrix(annot):
    import make_golden_matrix
    g = np.load(os.path.join(GOLD, "matrix_small.npz"), allow_pickle=False)
    r, o, l, idx, nidx = make_golden_matrix.matrix_inputs()
    assert make_golden.digest(r, o, l, idx) == str(g["input_sha256"]), "matrix fixture input drifted"
    assert nidx == int(g["n_idx"])
    return g, (r, o, l, idx, nidx)


def test_oracle_reproduces_matrix(annot, matrix):
    a, _ = annot
    g, (r, o, l, idx, nidx) = matrix
    funcs = list(a["functions"])
    ob = oracle_ref.Bdz(a["mph"].tobytes())
    got = oracle_ref.matrix_distance(ob, a["dat"].tobytes(), r, o, l, idx, funcs.index("hypothetical protein"))
    np.testing.assert_array_equal(got, g["pairs"])
    assert len(got) > 1000


@pytest.mark.gpu
def test_gpu_matrix_reproduces_golden(skm, gpu, annot, matrix):
    a, _ = annot
    g, (r, o, l, idx, nidx) = matrix
    db = skm.CmphKmerDb(mph=a["mph"].tobytes(), dat=a["dat"].tobytes(), device=gpu)
    md = skm.MatrixDistance(db, list(a["functions"]), r, o, l, seq_idx=idx, n_idx=nidx)
    np.testing.assert_array_equal(md.compute(), g["pairs"])
    md.close()
    db.close()


def test_multithreaded_annotate_port_counts_the_same_calls(annot):
    """oracle_annotate_mt (bench.py's all-core CPU baseline of the annotate leg) makes the calls
    of the single-thread restatement."""
    g, (qr, qo, ql) = annot
    funcs = list(g["functions"])
    ob = oracle_ref.Bdz(g["mph"].tobytes())
    hypo = funcs.index("hypothetical protein")
    for threads in (1, 3, 8):
        n = oracle_ref.annotate_mt(ob, g["dat"].tobytes(), qr, qo, ql, threads, hypo_index=hypo)
        assert n == len(g["calls"])
