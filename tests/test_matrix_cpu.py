"""CPU tests of the kmers-matrix-distance restatement (oracle/skm_oracle.cpp oracle_matrix_distance)
against an independent pure-Python restatement (pyref.matrix_distance) and hand-derived KATs of
hit_cb's length filter (kmers-matrix-distance.cc:132-149) and the set semantics of kmer_hit_map
(:121,151).  The DB is built with the host BDZ builder (CPU)."""
import numpy as np

import oracle_ref
import pyref
from signature_kmers_amd import synth


def pack(seqs):
    lens = np.array([len(s) for s in seqs], np.uint32)
    off = np.zeros(len(seqs), np.uint64)
    if len(seqs) > 1:
        off[1:] = np.cumsum(lens[:-1].astype(np.uint64))
    res = np.frombuffer(b"".join(seqs), np.uint8) if sum(map(len, seqs)) else np.zeros(0, np.uint8)
    return res, off, lens


def kmer(s: bytes) -> int:
    return int.from_bytes(s, "little")


def db_of(skm, tmp_path, recs):
    """recs: {kmer bytes: (avg, func, mean, median, var)} -> (Bdz, dat bytes, fetch)"""
    keys = np.array(sorted(kmer(k) for k in recs), np.uint64)
    byk = {kmer(k): v for k, v in recs.items()}
    data = np.array([byk[int(k)] for k in keys], oracle_ref.STORED_DTYPE)
    mph, dat = str(tmp_path / "m.mph"), str(tmp_path / "m.dat")
    skm.mph_build(keys, data, mph, dat, seed=5)
    bdz = oracle_ref.Bdz(open(mph, "rb").read())
    datb = open(dat, "rb").read()
    d = np.frombuffer(datb, oracle_ref.STORED_DTYPE)
    m = bdz.size()

    def fetch(key):  # CmphKmerDb::fetch: any key maps to some slot (no key check)
        i = int(bdz.search(np.array([key], np.uint64))[0])
        return tuple(int(x) for x in d[i]) if i < m else None
    return bdz, datb, fetch


def run_both(bdz, datb, fetch, seqs, idx, hypo):
    r, o, l = pack(seqs)
    got = oracle_ref.matrix_distance(bdz, datb, r, o, l, np.asarray(idx, np.uint32), hypo)
    exp = pyref.matrix_distance(seqs, idx, fetch, hypo)
    assert {(int(a), int(b)): int(c) for a, b, c in got} == exp
    assert np.all(np.diff(got[:, 0].astype(np.int64) * 2**32 + got[:, 1]) > 0) if len(got) > 1 else True
    return exp


def test_length_filter_kat(skm, tmp_path):
    # one signature k-mer per record kind; a sequence = filler of length L containing it
    K1, K2, K3 = b"ACDEFGHI", b"KLMNPQRS", b"TVWYACDE"
    recs = {K1: (0, 1, 100, 0, 0), K2: (0, 2, 100, 0, 16), K3: (0, 3, 100, 0, 15)}
    bdz, datb, fetch = db_of(skm, tmp_path, recs)

    def seq(k, L):
        # for_each_kmer yields only the k-mer: the window after it ends right before an 'X'
        # (skipped, kmer_data.h:90) and every later window contains one
        return k + b"W" + b"X" * (L - 9)
    # var == 0: keep iff 100 - 0.2 L <= L <= 100 + 0.2 L  ->  L in [84, 125]
    lens1 = [83, 84, 125, 126]
    # var == 16: sd = 4 -> [92, 108]; var == 15: sd = 3.873 -> [93, 107]
    lens2 = [91, 92, 108, 109]
    lens3 = [92, 93, 107, 108]
    seqs = [seq(K1, L) for L in lens1] + [seq(K2, L) for L in lens2] + [seq(K3, L) for L in lens3]
    exp = run_both(bdz, datb, fetch, seqs, list(range(len(seqs))), hypo=-1)
    # each kind: only the middle two lengths keep their hit -> exactly one pair per kind
    assert exp == {(1, 2): 1, (5, 6): 1, (9, 10): 1}


def test_sets_hypo_and_duplicate_ids(skm, tmp_path):
    K1, K2 = b"ACDEFGHI", b"KLMNPQRS"
    recs = {K1: (0, 1, 30, 0, 0), K2: (0, 7, 30, 0, 0)}
    bdz, datb, fetch = db_of(skm, tmp_path, recs)
    a = K1 + b"WX" + K1 + b"WX" + K2 + b"WX"     # K1 twice in one sequence: one set entry
    b = K2 + b"WX" + K1 + b"WX" + b"X" * 12
    # duplicate ids: sequences 0 and 2 share SeqIdMap index 0
    exp = run_both(bdz, datb, fetch, [a, b, a], [0, 1, 0], hypo=-1)
    assert exp == {(0, 1): 2}
    # function 7 is "hypothetical protein": its hits are dropped (ignore_hypothetical(true))
    exp = run_both(bdz, datb, fetch, [a, b, a], [0, 1, 0], hypo=7)
    assert exp == {(0, 1): 1}


def test_random_proteome_matches_pyref(skm, tmp_path):
    p = synth.generate_arrays(600, 12, per_file=200, seed=31)
    r, o, l, f, i, funcs = synth.build_inputs(p)
    ref = oracle_ref.build(r, o, l, f, i, len(funcs))
    mph, dat = str(tmp_path / "k.mph"), str(tmp_path / "k.dat")
    skm.mph_build(ref["keys"], ref["data"], mph, dat, seed=2)
    bdz = oracle_ref.Bdz(open(mph, "rb").read())
    datb = open(dat, "rb").read()
    d = np.frombuffer(datb, oracle_ref.STORED_DTYPE)
    q = synth.generate_arrays(1200, 12, per_file=200, first_file=3, n_files=1, seed=31, extras=True)
    seqs = [q.residues[q.seq_off[s]:q.seq_off[s] + q.seq_len[s]].tobytes() for s in range(len(q.seq_len))]
    seqs = seqs[:120]
    allk = sorted({k for s in seqs for _, k in pyref.call_windows(s)})
    slots = bdz.search(np.array(allk, np.uint64))
    table = {k: tuple(int(x) for x in d[sl]) for k, sl in zip(allk, slots) if sl < bdz.size()}
    hypo = funcs.index("hypothetical protein")
    exp = run_both(bdz, datb, table.get, seqs, list(range(len(seqs))), hypo)
    assert len(exp) > 100


def test_tile_rows_cover_and_balance(skm):
    """skm_matrix_tile_rows: the row bands of 1..8 GPUs cover [0, n) in order with nearly equal
    upper-triangle area (each GPU's share of the pair matrix)."""
    for n in (0, 1, 7, 1000, 100000):
        for world in (1, 2, 3, 4, 8):
            bands = [skm.matrix_tile_rows(n, r, world) for r in range(world)]
            assert bands[0][0] == 0 and bands[-1][1] == n
            for (a, b), (c, d) in zip(bands, bands[1:]):
                assert b == c and a <= b
            if n >= 1000:
                area = [sum(n - i - 1 for i in range(a, b)) for a, b in bands]
                assert max(area) - min(area) <= 2 * n, (n, world, area)  # one row of slack per band edge


def test_parallel_oracle_matrix_equals_single_thread():
    """oracle_matrix_distance_mt (bench.py's CPU baseline of the matrix leg) gives the
    single-thread restatement's pairs for any thread count."""
    from signature_kmers_amd import synth
    import tempfile
    import signature_kmers_amd as skm
    p = synth.generate_arrays(3000, 30, per_file=500, seed=9)
    r, o, l, f, i, funcs = synth.build_inputs(p)
    ref = oracle_ref.build(r, o, l, f, i, len(funcs))
    with tempfile.TemporaryDirectory() as d:
        base = d + "/kmer_data"
        skm.mph_build(ref["keys"], ref["data"], base + ".mph", base + ".dat", seed=1)
        ob = oracle_ref.Bdz(open(base + ".mph", "rb").read())
        dat = open(base + ".dat", "rb").read()
    q = synth.generate_arrays(5000, 30, per_file=500, first_file=6, n_files=4, seed=9)
    idx = (np.arange(len(q.seq_len)) % 1500).astype(np.uint32)  # repeated SeqIdMap indices too
    hypo = funcs.index("hypothetical protein")
    want = oracle_ref.matrix_distance(ob, dat, q.residues, q.seq_off, q.seq_len, idx, hypo)
    assert len(want) > 1000
    for t in (1, 3, 8):
        got = oracle_ref.matrix_distance_mt(ob, dat, q.residues, q.seq_off, q.seq_len, idx, hypo, n_threads=t)
        np.testing.assert_array_equal(got, want)
        assert oracle_ref.matrix_distance_mt(ob, dat, q.residues, q.seq_off, q.seq_len, idx, hypo, n_threads=t,
                                             want_pairs=False) == len(want)
