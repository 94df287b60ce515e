"""Host-side product code on the CPU: BDZ minimal-perfect-hash construction (build_perfect_hash,
perfect_hash.h:11-69), find_best_call (call_functions.tcc:347-659), function.index reading, and
the synthetic generator's determinism / shard independence.  Checked against the oracle."""
import os

import numpy as np
import pytest

import oracle_ref
from signature_kmers_amd import synth


# ------------------------------------------------------------------ BDZ construction (skm_bdz.cpp)
@pytest.mark.parametrize("n,seed", [(1, 1), (2, 3), (3, 5), (97, 7), (5000, 11), (200000, 13)])
def test_mph_build_is_minimal_perfect(skm, tmp_path, n, seed):
    rng = np.random.default_rng(n)
    keys = np.unique(rng.integers(0, 2**63, size=n + n // 10 + 4, dtype=np.uint64))[:n]
    rng.shuffle(keys)
    data = np.zeros(n, skm.STORED_DTYPE)
    for i, f in enumerate(skm.STORED_DTYPE.names):
        data[f] = rng.integers(0, 65536, size=n)
    mph, dat = str(tmp_path / "k.mph"), str(tmp_path / "k.dat")
    skm.mph_build(keys, data, mph, dat, seed=seed)
    img = open(mph, "rb").read()
    assert img[:4] == b"bdz\x00"                       # cmph_dump header
    ob = oracle_ref.Bdz(img)
    assert ob.size() == n
    idx = ob.search(keys)
    assert np.array_equal(np.sort(idx), np.arange(n, dtype=np.uint32))   # bijection onto [0, n)
    d = np.frombuffer(open(dat, "rb").read(), skm.STORED_DTYPE)
    assert len(d) == n
    np.testing.assert_array_equal(d[idx], data)       # perfect_hash.h:55-63 slot = search(key)


def test_mph_build_deterministic(skm, tmp_path):
    keys = np.arange(1, 3001, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
    data = np.zeros(len(keys), skm.STORED_DTYPE)
    a, b = str(tmp_path / "a"), str(tmp_path / "b")
    skm.mph_build(keys, data, a + ".mph", a + ".dat", seed=4)
    skm.mph_build(keys, data, b + ".mph", b + ".dat", seed=4)
    assert open(a + ".mph", "rb").read() == open(b + ".mph", "rb").read()


def test_mph_build_rejects_duplicates(skm, tmp_path):
    keys = np.array([5, 6, 5], np.uint64)
    with pytest.raises(skm.SkmError):
        skm.mph_build(keys, np.zeros(3, skm.STORED_DTYPE), str(tmp_path / "d.mph"), str(tmp_path / "d.dat"))


def test_jenkins_hash_is_seed_and_length_sensitive():
    a = oracle_ref.jenkins(1, b"ACDEFGHI")
    assert a != oracle_ref.jenkins(2, b"ACDEFGHI")
    assert a != oracle_ref.jenkins(1, b"ACDEFGHK")
    assert oracle_ref.jenkins(1, b"ACDEFGHI") == a


# ------------------------------------------------------------------ find_best_call (host C++)
FUNCS = sorted([f"function {i:05d}" for i in range(10)] +
               ["function 00001 / function 00003", "function 00005 / function 00002",
                "function 00007 / function 00001 / function 00004", "hypothetical protein"],
               key=lambda s: s.encode())


def mk_calls(rows):
    c = np.zeros(len(rows), oracle_ref.CALL_DTYPE)
    for j, (fi, cnt, med) in enumerate(rows):
        c[j] = (10 * j, 10 * j + 40, cnt, fi, 0, med, 1.5)
    return c


def check_same(rows):
    import signature_kmers_amd as skm
    c = mk_calls(rows)
    a = skm.find_best_call(c, FUNCS)
    b = oracle_ref.find_best_call(c, FUNCS)
    assert a[0] == b[0] and a[1] == b[1], (rows, a, b)
    assert np.float32(a[2]) == np.float32(b[2]) and np.float32(a[3]) == np.float32(b[3]), (rows, a, b)
    return a


def test_find_best_call_kats(skm):
    i = {f: k for k, f in enumerate(FUNCS)}
    f1, f3, f13 = i["function 00001"], i["function 00003"], i["function 00001 / function 00003"]
    # no calls -> undefined
    assert check_same([])[0] == 0xFFFF
    # single call: offset = its count; >= 5 calls it
    assert check_same([(f1, 7, 300)])[:2] == (f1, "function 00001")
    assert check_same([(f1, 4, 300)])[0] == 0xFFFF
    # fusion A W B with (a + b) ~ w -> the fusion (call_functions.tcc:526-553)
    r = check_same([(f1, 6, 200), (f13, 9, 500), (f3, 6, 300)])
    assert r[0] == f13 and r[2] == 21.0
    # lengths inconsistent with a fusion -> by-function sums (f13 9 vs 6 each)
    r = check_same([(f1, 6, 200), (f13, 9, 900), (f3, 6, 300)])
    assert r[0] == 0xFFFF or r[0] == f13
    # F1 F2 F1 merge when F2.count < 5 and F1+F1 >= 10 (:412-434), then a clear winner
    r = check_same([(f1, 6, 300), (f3, 2, 300), (f1, 6, 300)])
    assert r[0] == f1 and r[3] == 12.0   # the interior call is absorbed, not counted
    # close race -> "f1 ?? f2" fallback string (:633-657)
    r = check_same([(f1, 6, 300), (f3, 5, 300)])
    assert r[0] == 0xFFFF and "??" in r[1]


@pytest.mark.parametrize("seed", range(40))
def test_find_best_call_random_vs_oracle(skm, seed):
    rng = np.random.default_rng(seed)
    rows = []
    for _ in range(int(rng.integers(0, 9))):
        rows.append((int(rng.integers(0, len(FUNCS))), int(rng.integers(1, 25)), int(rng.integers(80, 1200))))
    if seed % 4 == 0 and len(rows) >= 3:   # plant a fusion pattern
        i = {f: k for k, f in enumerate(FUNCS)}
        a, b = int(rng.integers(150, 400)), int(rng.integers(150, 400))
        rows[:3] = [(i["function 00005"], 6, a), (i["function 00005 / function 00002"], 8, a + b + int(rng.integers(-40, 40))),
                    (i["function 00002"], 5, b)]
    check_same(rows)


# ------------------------------------------------------------------ function.index / generator
def test_read_function_index(skm, tmp_path):
    p = tmp_path / "function.index"
    p.write_bytes(b"0\talpha\t3\t1\t1\t0\t0\n2\tgamma / delta\t9\n1\tbeta\n")
    assert skm.read_function_index(str(p)) == ["alpha", "beta", "gamma / delta"]


def test_synth_is_deterministic_and_shardable():
    a = synth.generate_arrays(1200, 40, per_file=300)
    b = synth.generate_arrays(1200, 40, per_file=300)
    assert np.array_equal(a.residues, b.residues) and np.array_equal(a.labels, b.labels)
    # files [0,2) + [2,4) generated separately == files [0,4) (one RNG stream per file)
    s0 = synth.generate_arrays(1200, 40, per_file=300, first_file=0, n_files=2)
    s1 = synth.generate_arrays(1200, 40, per_file=300, first_file=2, n_files=2)
    assert np.array_equal(np.concatenate([s0.residues, s1.residues]), a.residues)
    assert np.array_equal(np.concatenate([s0.seq_len, s1.seq_len]), a.seq_len)
    r, o, l, f, i, funcs = synth.build_inputs(a)
    assert "hypothetical protein" in funcs and funcs == sorted(funcs, key=lambda s: s.encode())
    assert np.all(i[:300] == np.arange(300)) and np.all(i[300:600] == 100000 + np.arange(300))
    # ~330 mean length, 30 % trailing '*'
    assert 250 < l.mean() < 420
    ends = r[(o + l - 1).astype(np.int64)]
    assert 0.2 < np.mean(ends == ord("*")) < 0.4


def test_write_dirs_layout(tmp_path):
    info = synth.write_dirs(str(tmp_path), 250, 20, per_file=100)
    seqs = sorted(os.listdir(tmp_path / "Seqs"))
    anns = sorted(os.listdir(tmp_path / "Annotations"))
    assert seqs == anns and len(seqs) == 3
    txt = (tmp_path / "Seqs" / seqs[0]).read_text()
    assert txt.startswith(">fig|") and all(len(x) <= 60 for x in txt.splitlines() if not x.startswith(">"))
    assert isinstance(info, dict)


def _bdz_image(skm, tmp_path, n=1000):
    rng = np.random.default_rng(5)
    keys = np.unique(rng.integers(1, 2**63, size=n, dtype=np.uint64))
    data = np.zeros(len(keys), skm.STORED_DTYPE)
    base = str(tmp_path / "kmer_data")
    skm.mph_build(keys, data, base + ".mph", base + ".dat", seed=1)  # host construction
    return bytearray(open(base + ".mph", "rb").read()), open(base + ".dat", "rb").read()


def test_malformed_bdz_images_are_rejected_before_any_device_use(skm, tmp_path):
    """bdz_parse bounds every index the searches use: n = 3r (64-bit), m <= n, b < 32,
    k = 2^b, ranktablesize >= ceil(n/k).  A bad image fails with the parse error; a good one
    gets past parsing (and then fails only for want of a device here)."""
    import ctypes as C
    lib = skm.lib()
    img, dat = _bdz_image(skm, tmp_path)
    n = int.from_bytes(img[24:28], "little")
    koff = 36 + (n + 3) // 4

    def open_err(buf):
        h = C.c_void_p()
        b = bytes(buf)
        rc = lib.skm_db_open_mem(C.byref(h), b, len(b), dat, len(dat), 0)
        return rc, lib.skm_last_error().decode()

    rc, msg = open_err(img)
    assert "kmer_data.mph" not in msg  # parsed fine; any failure here is the missing device
    bad = []
    x = bytearray(img); x[32:36] = (0x55555556).to_bytes(4, "little"); bad.append(x)   # 3r wraps to n in u32
    x = bytearray(img); x[koff + 4] = 40; bad.append(x)                                # b >= 32
    x = bytearray(img); x[koff:koff + 4] = (64).to_bytes(4, "little"); bad.append(x)    # k != 2^b
    x = bytearray(img); x[koff + 5:koff + 9] = (1).to_bytes(4, "little"); bad.append(x[:koff + 13])  # short rank table
    x = bytearray(img); x[4:8] = (n + 1).to_bytes(4, "little"); x[28:32] = (n + 1).to_bytes(4, "little"); bad.append(x)  # m > n
    for b in bad:
        rc, msg = open_err(b)
        assert rc != 0 and "kmer_data.mph" in msg, msg


# function names that stress split(" / ") in the fusion keys (call_functions.tcc:487;
# split itself is pinned against the reference in test_ref_pin_cpu.py)
FUNCS_SPLIT = sorted(["alpha", "beta", "alpha / beta", "alpha / ", " / beta", "alpha / / beta", "x // y",
                      "alpha /  / beta", "beta / alpha", "alpha / beta / ", "a/b", "hypothetical protein", ""],
                     key=lambda s: s.encode())


@pytest.mark.parametrize("seed", range(30))
def test_find_best_call_split_edge_names_vs_oracle(skm, seed):
    import signature_kmers_amd as skm_pkg
    rng = np.random.default_rng(1000 + seed)
    rows = [(int(rng.integers(0, len(FUNCS_SPLIT))), int(rng.integers(1, 15)), int(rng.integers(80, 900)))
            for _ in range(int(rng.integers(1, 7)))]
    if seed % 3 == 0:  # A W B shaped around the edge names
        i = {f: k for k, f in enumerate(FUNCS_SPLIT)}
        w = ["alpha / beta", "alpha / / beta", "alpha / ", " / beta"][seed % 4]
        rows = [(i["alpha"], 6, 200), (i[w], 9, 500), (i["beta"], 6, 300)] + rows[:2]
    c = mk_calls(rows)
    a = skm_pkg.find_best_call(c, FUNCS_SPLIT)
    b = oracle_ref.find_best_call(c, FUNCS_SPLIT)
    assert a[0] == b[0] and a[1] == b[1], (rows, a, b)
    assert np.float32(a[2]) == np.float32(b[2]) and np.float32(a[3]) == np.float32(b[3]), (rows, a, b)
