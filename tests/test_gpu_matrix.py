"""GPU parity: kmers-matrix-distance pair counts (skm_matrix_*) vs the CPU oracle
(oracle_matrix_distance, pinned by test_matrix_cpu.py), bit-exact as sorted (id1, id2, count)."""
import numpy as np
import pytest

import oracle_ref
from signature_kmers_amd import synth

pytestmark = pytest.mark.gpu


def make_db(skm, tmp_path, n_seqs=3000, fam=30, seed=41):
    p = synth.generate_arrays(n_seqs, fam, per_file=500, seed=seed)
    r, o, l, f, i, funcs = synth.build_inputs(p)
    ref = oracle_ref.build(r, o, l, f, i, len(funcs))
    base = str(tmp_path / "kmer_data")
    skm.mph_build(ref["keys"], ref["data"], base + ".mph", base + ".dat", seed=7)
    return ref, funcs, base


def queries(n, fam=30, seed=41, first_file=20, per_file=500, extras=True):
    nf = (n + per_file - 1) // per_file
    return synth.generate_arrays((first_file + nf) * per_file, fam, per_file=per_file, first_file=first_file,
                                 n_files=nf, seed=seed, extras=extras)


def oracle_pairs(base, funcs, q, idx):
    ob = oracle_ref.Bdz(open(base + ".mph", "rb").read())
    return oracle_ref.matrix_distance(ob, open(base + ".dat", "rb").read(), q.residues, q.seq_off, q.seq_len,
                                      idx, funcs.index("hypothetical protein"))


def test_matrix_matches_oracle(skm, gpu, tmp_path):
    ref, funcs, base = make_db(skm, tmp_path)
    db = skm.CmphKmerDb(base)
    q = queries(1500)
    md = skm.MatrixDistance(db, funcs, q.residues, q.seq_off, q.seq_len)
    got = md.compute()
    exp = oracle_pairs(base, funcs, q, np.arange(len(q.seq_len), dtype=np.uint32))
    assert len(exp) > 10000
    np.testing.assert_array_equal(got, exp)
    c = md.counters()
    assert c["pairs"] == len(exp) and c["increments"] == int(exp[:, 2].sum())
    # re-run on the resident queries: the tile was reset by the compaction
    np.testing.assert_array_equal(md.compute(), exp)
    md.close()
    db.close()


def test_matrix_tiles_and_bands(skm, gpu, tmp_path):
    """Row tiles of 3 'GPUs' (equal triangle area) and row bands forced by a small tile budget
    concatenate to the full matrix."""
    ref, funcs, base = make_db(skm, tmp_path)
    db = skm.CmphKmerDb(base)
    q = queries(1000, first_file=30)
    md = skm.MatrixDistance(db, funcs, q.residues, q.seq_off, q.seq_len)
    full = md.compute()
    n = len(q.seq_len)
    parts = []
    for r in range(3):
        a, b = skm.matrix_tile_rows(n, r, 3)
        t = md.compute(rows=(a, b))
        assert len(t) == 0 or (t[:, 0].min() >= a and t[:, 0].max() < b)
        parts.append(t)
    np.testing.assert_array_equal(np.concatenate(parts), full)
    md.run(max_tile_bytes=64 * 1024)  # ~ a few rows per band
    np.testing.assert_array_equal(md.pairs(), full)
    md.close()
    db.close()


def test_matrix_duplicate_ids_and_edges(skm, gpu, tmp_path):
    ref, funcs, base = make_db(skm, tmp_path, n_seqs=1500, fam=20, seed=9)
    db = skm.CmphKmerDb(base)
    q = queries(400, fam=20, seed=9, first_file=10, per_file=200)
    seqs = [q.residues[q.seq_off[s]:q.seq_off[s] + q.seq_len[s]].tobytes() for s in range(len(q.seq_len))]
    src = seqs[0]
    seqs += [b"", b"ACDEFGH", b"ACDEFGHI", b"XXXXXXXXXX", src, src, src.lower(), src[:30] + b"X" + src[30:],
             src * 5, b"*" + src + b"*"]
    lens = np.array([len(s) for s in seqs], np.uint32)
    off = np.zeros(len(seqs), np.uint64)
    off[1:] = np.cumsum(lens[:-1].astype(np.uint64))
    res = np.frombuffer(b"".join(seqs), np.uint8)
    # SeqIdMap: every 7th sequence repeats the id of the sequence 3 before it
    ids = skm.SeqIdMap()
    names = [f"fig|1.1.peg.{s}" for s in range(len(seqs))]
    for s in range(7, len(seqs), 7):
        names[s] = names[s - 3]
    idx = np.array([ids.lookup_id(nm) for nm in names], np.uint32)
    md = skm.MatrixDistance(db, funcs, res, off, lens, seq_idx=idx, n_idx=len(ids))
    got = md.compute()

    class Q:
        pass
    qq = Q()
    qq.residues, qq.seq_off, qq.seq_len = res, off, lens
    exp = oracle_pairs(base, funcs, qq, idx)
    np.testing.assert_array_equal(got, exp)
    md.close()
    # no sequences at all
    md = skm.MatrixDistance(db, funcs, np.zeros(0, np.uint8), np.zeros(0, np.uint64), np.zeros(0, np.uint32))
    assert md.compute().shape == (0, 3)
    md.close()
    db.close()


def test_matrix_exact_db(skm, gpu, tmp_path):
    """Against the exact kept-k-mer DB (KeptKmerDB semantics: only real signature k-mers hit)."""
    ref, funcs, base = make_db(skm, tmp_path, n_seqs=2000, fam=20, seed=13)
    db = skm.KeptKmerDb(ref["keys"], ref["data"])
    q = queries(800, fam=20, seed=13, first_file=12, per_file=400)
    md = skm.MatrixDistance(db, funcs, q.residues, q.seq_off, q.seq_len)
    got = md.compute()
    # oracle: exact fetch == BDZ fetch restricted to member keys; restate through pyref
    import pyref
    keys = {int(k): tuple(int(x) for x in d) for k, d in zip(ref["keys"], ref["data"])}
    seqs = [q.residues[q.seq_off[s]:q.seq_off[s] + q.seq_len[s]].tobytes() for s in range(len(q.seq_len))]
    exp = pyref.matrix_distance(seqs, list(range(len(seqs))), keys.get, funcs.index("hypothetical protein"))
    assert {(int(a), int(b)): int(c) for a, b, c in got} == exp
    assert len(exp) > 1000
    md.close()
    db.close()


def test_c5_full_100k_bit_exact(skm, gpu, tmp_path):
    """BASELINE configs[4] at full size, the bench's matrix leg: a 200-family signature DB built on
    the GPU from 200K training proteins (genome files 0..49, device-peeled BDZ), all-vs-all over
    the 100K fresh query proteins of files 50..74 (~73M nonzero pairs, ~293M pair increments) vs
    oracle_matrix_distance on every host core (kmers-matrix-distance.cc:123-211), bit-exact as
    sorted (id1, id2, count)."""
    import os
    fam, per = 200, 4000
    th = len(os.sched_getaffinity(0))
    try:
        qq, pp = open("/sys/fs/cgroup/cpu.max").read().split()
        if qq != "max":
            th = max(1, min(th, int(qq) // int(pp)))
    except (OSError, ValueError):
        pass

    def packed(n_total, f0, nf):
        parts = list(synth.iter_file_inputs(n_total, fam, per, f0, nf, workers=min(16, th)))
        cat = [np.concatenate([p[k] for p in parts]) for k in range(5)]
        off = np.zeros(len(cat[2]), np.uint64)
        off[1:] = np.cumsum(cat[2][:-1], dtype=np.uint64)
        return cat[0], off, cat[2], cat[3], cat[4]

    funcs = synth.functions(fam)
    r, o, l, f, i = packed(200_000, 0, 50)
    b = skm.SignatureBuilder(len(funcs))
    b.add_batch(r, o, l, f, i)
    kept = b.finish()
    b.close()
    base = str(tmp_path / "kmer_data")
    skm.mph_build(kept.keys, kept.data, base + ".mph", base + ".dat", seed=1, device=0)
    qr, qo, ql, _, _ = packed(300_000, 50, 25)
    assert len(ql) == 100_000
    db = skm.CmphKmerDb(base, device=0)
    md = skm.MatrixDistance(db, funcs, qr, qo, ql)
    got = md.compute()
    c = md.counters()
    md.close()
    db.close()
    ob = oracle_ref.Bdz(open(base + ".mph", "rb").read())
    exp = oracle_ref.matrix_distance_mt(ob, open(base + ".dat", "rb").read(), qr, qo, ql,
                                        np.arange(len(ql), dtype=np.uint32), funcs.index("hypothetical protein"),
                                        n_threads=th)
    assert len(exp) > 50_000_000, len(exp)
    assert c["pairs"] == len(exp) and c["increments"] == int(exp[:, 2].astype(np.int64).sum())
    assert np.array_equal(got, exp)
