"""GPU parity: HBM-resident CMPH/BDZ lookup and the HitSet call path vs the CPU oracle."""
import os

import numpy as np
import pytest

import oracle_ref
from signature_kmers_amd import synth

pytestmark = pytest.mark.gpu


def make_db(skm, tmp_path, n_seqs=3000, fam=60, seed=21):
    p = synth.generate_arrays(n_seqs, fam, per_file=500, seed=seed)
    r, o, l, f, i, funcs = synth.build_inputs(p)
    ref = oracle_ref.build(r, o, l, f, i, len(funcs))
    mph = str(tmp_path / "kmer_data.mph")
    dat = str(tmp_path / "kmer_data.dat")
    skm.mph_build(ref["keys"], ref["data"], mph, dat, seed=7)
    return ref, funcs, mph, dat, p


def test_lookup_members_and_strangers(skm, gpu, tmp_path):
    ref, funcs, mph, dat, _ = make_db(skm, tmp_path)
    db = skm.CmphKmerDb(str(tmp_path / "kmer_data"))
    m = db.hash_size()
    assert m == len(ref["keys"])
    idx = db.lookup_keys(ref["keys"])
    assert np.array_equal(np.sort(idx), np.arange(m, dtype=np.uint32))  # minimal perfect
    ob = oracle_ref.Bdz(open(mph, "rb").read())
    np.testing.assert_array_equal(idx, ob.search(ref["keys"]))
    rng = np.random.default_rng(3)
    strangers = rng.integers(0, 2**63, size=200000, dtype=np.uint64)
    np.testing.assert_array_equal(db.lookup_keys(strangers), ob.search(strangers))
    # the .dat slot of each member holds its record
    d = np.frombuffer(open(dat, "rb").read(), dtype=skm.STORED_DTYPE)
    np.testing.assert_array_equal(d[idx], ref["data"])


@pytest.mark.parametrize("n", [1, 2, 41, 42, 43, 127, 128, 129, 1000, 4099, 65537])
def test_pair_line_lookup_matches_bdz_search(skm, gpu, tmp_path, n):
    """The b = 7 (g word, rank) pair-line search (bdz7_lookup: skm_db_lookup, k_lookup<0>, the
    matrix hits) equals cmph bdz_search (oracle) and the generic device walk, per key, for members
    and strangers.  Key counts put the last vertex block anywhere from one pair to a full line
    (the padded final block); 400K strangers hit every vertex of these hashes, so every pair,
    word and 128-vertex line boundary is exercised."""
    rng = np.random.default_rng(1000 + n)
    keys = np.unique(rng.integers(1, 2**63, size=n, dtype=np.uint64))
    data = np.zeros(len(keys), skm.STORED_DTYPE)
    data["function_index"] = np.arange(len(keys)) % 4000
    base = str(tmp_path / "kmer_data")
    skm.mph_build(keys, data, base + ".mph", base + ".dat", seed=7)
    ob = oracle_ref.Bdz(open(base + ".mph", "rb").read())
    db = skm.CmphKmerDb(base)
    strangers = rng.integers(0, 2**64 - 1, size=400000, dtype=np.uint64)
    for q in (keys, strangers):
        want = ob.search(q)
        np.testing.assert_array_equal(db.lookup_keys(q), want)
        np.testing.assert_array_equal(db.lookup_keys_generic(q), want)
    assert np.array_equal(np.sort(db.lookup_keys(keys)), np.arange(len(keys), dtype=np.uint32))
    db.close()


@pytest.mark.parametrize("ignore_hypo", [0, 1])
def test_calls_match_oracle(skm, gpu, tmp_path, ignore_hypo):
    ref, funcs, mph, dat, _ = make_db(skm, tmp_path)
    db = skm.CmphKmerDb(str(tmp_path / "kmer_data"))
    caller = skm.FunctionCaller(db, funcs)
    caller.ignore_hypothetical(bool(ignore_hypo))
    # fresh queries from the same families (files the DB never saw)
    q = synth.generate_arrays(100000, 60, per_file=500, first_file=40, n_files=8, seed=21, extras=True)
    off, calls = caller.process_seqs(q.residues, q.seq_off, q.seq_len)
    ob = oracle_ref.Bdz(open(mph, "rb").read())
    ooff, ocalls = oracle_ref.annotate(ob, open(dat, "rb").read(), q.residues, q.seq_off, q.seq_len,
                                       ignore_hypo=ignore_hypo, hypo_index=funcs.index("hypothetical protein"))
    np.testing.assert_array_equal(off, ooff)
    assert len(calls) == len(ocalls) and len(calls) > 100
    for f in ("start", "end", "count", "function_index", "protein_length_median"):
        np.testing.assert_array_equal(calls[f], ocalls[f], err_msg=f)
    np.testing.assert_array_equal(calls["protein_length_med_avg_dev"].view(np.uint32),
                                  ocalls["protein_length_med_avg_dev"].view(np.uint32))
    # host find_best_call (product) == oracle find_best_call
    n_called = 0
    for s in range(len(q.seq_len)):
        c = calls[off[s]:off[s + 1]]
        a = caller.find_best_call(c)
        b = oracle_ref.find_best_call(c, funcs)
        assert a[0] == b[0] and a[1] == b[1] and a[2] == b[2], (s, a, b)
        n_called += a[0] != 0xFFFF
    assert n_called > len(q.seq_len) // 2


def test_query_edge_cases(skm, gpu, tmp_path):
    ref, funcs, mph, dat, p = make_db(skm, tmp_path, n_seqs=1500, fam=30, seed=5)
    db = skm.CmphKmerDb(str(tmp_path / "kmer_data"))
    caller = skm.FunctionCaller(db, funcs)
    src = p.residues[p.seq_off[0]:p.seq_off[0] + p.seq_len[0]].tobytes()
    seqs = [b"", b"ACDEFGH", b"ACDEFGHI", b"ACDEFGHIX", b"XACDEFGHI", src, src[:50] + b"X" + src[50:],
            src[:40] + b"*" + src[41:], src.lower(), src * 3, b"X" * 20, src * 7, src * 12, src * 40]
    lens = np.array([len(s) for s in seqs], np.uint32)
    off = np.zeros(len(seqs), np.uint64)
    off[1:] = np.cumsum(lens[:-1])
    res = np.frombuffer(b"".join(seqs), np.uint8)
    goff, gcalls = caller.process_seqs(res, off, lens)
    ob = oracle_ref.Bdz(open(mph, "rb").read())
    ooff, ocalls = oracle_ref.annotate(ob, open(dat, "rb").read(), res, off, lens,
                                       hypo_index=funcs.index("hypothetical protein"))
    np.testing.assert_array_equal(goff, ooff)
    np.testing.assert_array_equal(gcalls.view(np.uint8), ocalls.view(np.uint8))


@pytest.mark.parametrize("kind", ["exact", "bdz"])
def test_device_windows_match_reference(skm, gpu, tmp_path, kind):
    """The device window iterator (k_lookup's validity test: no 'X' / '*' in the window or the byte
    right after it) against the REFERENCE's own for_each_kmer<8> (kmer_data.h:76-102, compiled
    from the reference: tests/golden/ref_windows.npz).  The DB holds every k-mer of every valid
    window, so the device's hit windows (skm_query_window_hits) are exactly its windows."""
    from test_ref_pin_cpu import ref_windows
    seqs, wins = ref_windows()
    keys = [int.from_bytes(s[q:q + 8], "little") for s, w in zip(seqs, wins) for q in w]
    keys = np.unique(np.array(keys, np.uint64))
    data = np.zeros(len(keys), skm.STORED_DTYPE)
    data["function_index"] = 1 + np.arange(len(keys)) % 7
    data["mean"] = np.arange(len(keys)) % 60000
    if kind == "exact":
        db = skm.KeptKmerDb(keys, data)
    else:
        base = str(tmp_path / "kmer_data")
        skm.mph_build(keys, data, base + ".mph", base + ".dat", seed=3)
        db = skm.CmphKmerDb(base)
    lens = np.array([len(s) for s in seqs], np.uint32)
    off = np.zeros(len(seqs), np.uint64)
    off[1:] = np.cumsum(lens[:-1])
    qb = skm.QueryBatch(db, np.frombuffer(b"".join(seqs), np.uint8), off, lens)
    qb.run(hypo_index=-1)
    hoff, pos, fm = qb.window_hits()
    for i, w in enumerate(wins):
        np.testing.assert_array_equal(pos[hoff[i]:hoff[i + 1]], w.astype(np.uint32), err_msg=repr(seqs[i]))
    # each hit carries its own record's function_index << 16 | mean
    got = np.array([int.from_bytes(seqs[i][q:q + 8], "little") for i in range(len(seqs))
                    for q in pos[hoff[i]:hoff[i + 1]]], np.uint64)
    j = np.searchsorted(keys, got)
    want = (data["function_index"][j].astype(np.uint32) << 16) | data["mean"][j]
    if kind == "exact":
        np.testing.assert_array_equal(fm, want)
    else:
        slot = db.lookup_keys(got)
        d = np.frombuffer(open(str(tmp_path / "kmer_data.dat"), "rb").read(), skm.STORED_DTYPE)
        np.testing.assert_array_equal(fm, (d["function_index"][slot].astype(np.uint32) << 16) | d["mean"][slot])
        np.testing.assert_array_equal(fm, want)
    qb.close()
    db.close()


def test_kept_db_exact_lookup_and_recall_calls(skm, gpu, tmp_path):
    """KeptKmerDB (exact keys): members hit their own record, strangers miss; the call path over
    it equals the oracle's recall-pass restatement (kept_kmer_db.h:20-27)."""
    ref, funcs, _, _, p = make_db(skm, tmp_path, n_seqs=2000, fam=50, seed=5)
    db = skm.KeptKmerDb(ref["keys"], ref["data"])
    n = len(ref["keys"])
    assert db.hash_size() == n
    np.testing.assert_array_equal(db.lookup_keys(ref["keys"]), np.arange(n, dtype=np.uint32))
    rng = np.random.default_rng(11)
    strangers = rng.integers(1, 2**63, size=100000, dtype=np.uint64)
    strangers = strangers[~np.isin(strangers, ref["keys"])]
    assert (db.lookup_keys(strangers) == n).all()
    hypo = funcs.index("hypothetical protein")
    caller = skm.FunctionCaller(db, funcs)
    off, calls = caller.process_seqs(p.residues, p.seq_off, p.seq_len)
    ooff, ocalls = oracle_ref.annotate_exact(ref["keys"], ref["data"], p.residues, p.seq_off, p.seq_len,
                                             hypo_index=hypo)
    assert len(calls) > 100
    np.testing.assert_array_equal(off, ooff)
    np.testing.assert_array_equal(calls.view(np.uint8), ocalls.view(np.uint8))
    empty = skm.KeptKmerDb(np.zeros(0, np.uint64), np.zeros(0, skm.STORED_DTYPE))
    assert (empty.lookup_keys(ref["keys"][:10]) == 0).all()


@pytest.mark.parametrize("n", [1500, 300000])
def test_device_mph_build_is_minimal_perfect(skm, gpu, tmp_path, n):
    """skm_mph_build_device: the GPU-peeled BDZ image is cmph-readable (oracle reader), minimal
    perfect over the keys, places every record, and is deterministic for a seed."""
    rng = np.random.default_rng(n)
    keys = np.unique(rng.integers(1, 2**63, size=n, dtype=np.uint64))
    rng.shuffle(keys)
    data = np.zeros(len(keys), skm.STORED_DTYPE)
    data["function_index"] = np.arange(len(keys)) % 65000
    data["avg_from_end"] = np.arange(len(keys)) // 7
    mph, dat = str(tmp_path / "a.mph"), str(tmp_path / "a.dat")
    skm.mph_build(keys, data, mph, dat, seed=3, device=0)
    ob = oracle_ref.Bdz(open(mph, "rb").read())
    assert ob.size() == len(keys)
    idx = ob.search(keys)
    assert np.array_equal(np.sort(idx), np.arange(len(keys), dtype=np.uint32))
    d = np.frombuffer(open(dat, "rb").read(), skm.STORED_DTYPE)
    assert np.array_equal(d[idx].view(np.uint8), data.view(np.uint8))
    skm.mph_build(keys, data, str(tmp_path / "b.mph"), str(tmp_path / "b.dat"), seed=3, device=0)
    assert open(mph, "rb").read() == open(str(tmp_path / "b.mph"), "rb").read()
    db = skm.CmphKmerDb(str(tmp_path / "a"))
    np.testing.assert_array_equal(db.lookup_keys(keys), idx)


def test_device_mph_build_ex_verifies_and_matches(skm, gpu, tmp_path):
    """skm_mph_build_device_ex: the same image as skm_mph_build_device; its on-device check
    passes; NULL paths build and check without writing; duplicate keys are refused."""
    rng = np.random.default_rng(11)
    keys = np.unique(rng.integers(1, 2**63, size=400000, dtype=np.uint64))  # ascending
    data = np.zeros(len(keys), skm.STORED_DTYPE)
    data["function_index"] = np.arange(len(keys)) % 50000
    data["var"] = np.arange(len(keys)) % 65521
    a, b = str(tmp_path / "a"), str(tmp_path / "b")
    skm.mph_build(keys, data, a + ".mph", a + ".dat", seed=5, device=0)
    st = skm.mph_build_device(keys, data, b + ".mph", b + ".dat", seed=5, device=0, verify=True)
    assert st["verified"] == 1 and st["n_keys"] == len(keys) and st["attempts"] >= 1 and st["peel_rounds"] > 0
    assert st["n_vertices"] >= 1.23 * len(keys) - 3
    assert open(a + ".mph", "rb").read() == open(b + ".mph", "rb").read()
    assert open(a + ".dat", "rb").read() == open(b + ".dat", "rb").read()
    st2 = skm.mph_build_device(keys, data, None, None, seed=5, device=0, verify=True)
    assert st2["verified"] == 1 and st2["n_vertices"] == st["n_vertices"]
    dup = keys.copy()
    dup[1000] = dup[999]
    with pytest.raises(skm.SkmError):
        skm.mph_build_device(dup, data, None, None, seed=5, device=0)


def _long_family(rng, n_copies, length, func, first_id):
    """n_copies ~1 %-mutated variants of one random protein of `length` residues, one function:
    their k-mers are kept with a mean length near `length`, so a query of that length makes a
    call whose segment has > 1024 hits (the sequential HitSet path)."""
    aa = np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY", np.uint8)
    base = aa[rng.integers(0, 20, length)]
    seqs = []
    for _ in range(n_copies):
        v = base.copy()
        m = rng.random(length) < 0.01
        v[m] = aa[rng.integers(0, 20, int(m.sum()))]
        seqs.append(v)
    lens = np.full(n_copies, length, np.uint32)
    return seqs, lens, np.full(n_copies, func, np.uint16), np.arange(first_id, first_id + n_copies, dtype=np.uint32)


@pytest.mark.parametrize("mean_mode,mad_mode", [(1, 0), (0, 1), (1, 1)])
def test_boost_math_modes_match_oracle(skm, gpu, tmp_path, mean_mode, mad_mode):
    """The Boost.Math switch (call_functions.tcc:51-53) on the device: the single
    running mean (mean_mode 1) and the older MAD returning |x(mid)| after libstdc++'s nth_element
    permutations (mad_mode 1) equal the oracle (std::nth_element itself), on the LDS segment path
    and on the > 1024-hit sequential path (a long protein family added to the DB)."""
    rng = np.random.default_rng(77)
    p = synth.generate_arrays(3000, 60, per_file=500, seed=21)
    r, o, l, f, i, funcs = synth.build_inputs(p)
    lseqs, llens, lf, lid = _long_family(rng, 14, 3000, int(f[f != 0xFFFF][0]), int(i.max()) + 1)
    r2 = np.concatenate([r] + lseqs)
    o2 = np.concatenate([o, len(r) + np.arange(len(lseqs), dtype=np.uint64) * 3000])
    ref = oracle_ref.build(r2, o2, np.concatenate([l, llens]), np.concatenate([f, lf]), np.concatenate([i, lid]),
                           len(funcs))
    base = str(tmp_path / "kmer_data")
    skm.mph_build(ref["keys"], ref["data"], base + ".mph", base + ".dat", seed=7)
    db = skm.CmphKmerDb(base)
    q = synth.generate_arrays(60000, 60, per_file=500, first_file=40, n_files=6, seed=21, extras=True)
    seqs = [q.residues[q.seq_off[k]:q.seq_off[k] + q.seq_len[k]].tobytes() for k in range(len(q.seq_len))]
    seqs += [v.tobytes() for v in lseqs[:6]]
    lens = np.array([len(s) for s in seqs], np.uint32)
    off = np.zeros(len(seqs), np.uint64)
    off[1:] = np.cumsum(lens[:-1])
    res = np.frombuffer(b"".join(seqs), np.uint8)
    hypo = funcs.index("hypothetical protein")
    caller = skm.FunctionCaller(db, funcs, mean_mode=mean_mode, mad_mode=mad_mode)
    goff, gcalls = caller.process_seqs(res, off, lens)
    ob = oracle_ref.Bdz(open(base + ".mph", "rb").read())
    dat = open(base + ".dat", "rb").read()
    ooff, ocalls = oracle_ref.annotate(ob, dat, res, off, lens, hypo_index=hypo, mean_mode=mean_mode,
                                       mad_mode=mad_mode)
    assert len(gcalls) > 1000 and (gcalls["count"] > 1024).any()
    np.testing.assert_array_equal(goff, ooff)
    np.testing.assert_array_equal(gcalls.view(np.uint8), ocalls.view(np.uint8))
    if mad_mode:  # the switch changes results on this data (ties in |x - median| are common)
        _, base_calls = oracle_ref.annotate(ob, dat, res, off, lens, hypo_index=hypo, mean_mode=mean_mode, mad_mode=0)
        assert len(base_calls) != len(ocalls) or not np.array_equal(base_calls.view(np.uint8), ocalls.view(np.uint8))


@pytest.mark.parametrize("span", [1024, 1025, 65536])
def test_calls_wide_length_spans(skm, gpu, tmp_path, span):
    """The HitSet median / MAD over segments whose k-mer mean lengths span up to `span` values
    (call_functions.tcc:35-103): k_seg_process takes its LDS histograms when a segment's values
    span <= 1024 and the wave radix selects above; the .dat means are rewritten with random values
    in [300, 300 + span) so both paths and the boundary between them run, compared with the
    oracle bit for bit."""
    ref, funcs, mph, dat, _ = make_db(skm, tmp_path, n_seqs=2000, fam=40, seed=9)
    d = np.frombuffer(open(dat, "rb").read(), dtype=skm.STORED_DTYPE).copy()
    rng = np.random.default_rng(span)
    d["mean"] = (300 + rng.integers(0, span, size=len(d))).clip(0, 65535).astype(np.uint16)
    open(dat, "wb").write(d.tobytes())
    db = skm.CmphKmerDb(str(tmp_path / "kmer_data"))
    caller = skm.FunctionCaller(db, funcs)
    q = synth.generate_arrays(20000, 40, per_file=500, first_file=40, n_files=4, seed=23, extras=True)
    goff, gcalls = caller.process_seqs(q.residues, q.seq_off, q.seq_len)
    ob = oracle_ref.Bdz(open(mph, "rb").read())
    ooff, ocalls = oracle_ref.annotate(ob, open(dat, "rb").read(), q.residues, q.seq_off, q.seq_len,
                                       hypo_index=funcs.index("hypothetical protein"))
    np.testing.assert_array_equal(goff, ooff)
    assert len(gcalls) == len(ocalls)
    np.testing.assert_array_equal(gcalls.view(np.uint8), ocalls.view(np.uint8))
    db.close()
