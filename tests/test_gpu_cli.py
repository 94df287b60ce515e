"""GPU tests of the drop-in CLIs (bin/kmers-build-signatures, kmers-call-functions,
kmers-annotate-seqs) end to end against the oracle: every output file of the reference mains,
byte for byte (final.kmers / distinct_functions compared as line sets: the reference writes them
in hash-table order)."""
import os
import subprocess

import numpy as np
import pytest

import front_data
import oracle_ref
from conftest import ROOT

import oracle.front_ref as fr  # noqa: E402  (test infrastructure)

BIN = os.path.join(ROOT, "bin")
pytestmark = pytest.mark.gpu


def _lines(path):
    with open(path, "rb") as fh:
        return fh.read()


def _fidx(out):
    t = []
    for line in _lines(os.path.join(out, "function.index")).split(b"\n"):
        if line:
            c = line.split(b"\t")
            i = int(c[0])
            t += [""] * (i + 1 - len(t))
            t[i] = c[1].decode("latin-1")
    return t


def _parse_final_kmers(buf: bytes):
    """final.kmers (kmers-build-signatures.cc:212-216: KMER \t avg_from_end \t function_index \t \n,
    the key as its 8 raw residue bytes) -> (u64 little-endian keys, avg, fi), in file order; every
    line must have exactly that shape."""
    b = np.frombuffer(buf, np.uint8)
    if len(b) == 0:
        return np.zeros(0, np.uint64), np.zeros(0, np.uint16), np.zeros(0, np.uint16)
    assert b[-1] == 10
    nl = np.flatnonzero(b == 10)
    starts = np.concatenate([[0], nl[:-1] + 1])
    keys = np.zeros(len(starts), np.uint64)
    for j in range(8):
        keys |= b[starts + j].astype(np.uint64) << np.uint64(8 * j)
    tabs = np.flatnonzero(b == 9)
    assert len(tabs) == 3 * len(starts)
    tabs = tabs.reshape(-1, 3)
    assert np.array_equal(tabs[:, 0], starts + 8) and np.array_equal(tabs[:, 2], nl - 1)

    def field(lo, hi):  # decimal digits in (lo, hi)
        w = hi - lo - 1
        assert w.min() >= 1 and w.max() <= 5
        v = np.zeros(len(lo), np.int64)
        for d in range(5):
            i = hi - 1 - d
            ok = i > lo
            dig = b[np.where(ok, i, lo)].astype(np.int64) - 48
            assert np.all((dig[ok] >= 0) & (dig[ok] <= 9))
            v += np.where(ok, dig * 10 ** d, 0)
        return v.astype(np.uint16)
    return keys, field(tabs[:, 0], tabs[:, 1]), field(tabs[:, 1], tabs[:, 2])


def _check_build(out, stdout, ref, threads=0, report_stride=1):
    """Every output of kmers-build-signatures vs the oracle; threads > 0: the oracle build on that
    many host threads (oracle_build_mt) and the recall reports' files in parallel; report_stride:
    the recall reports of every report_stride-th file (their restatement is per-record Python)."""
    res, off, ln, fn, sid = ref["build"]
    nf = ref["n_kept_functions"]
    o = oracle_ref.build_mt(res, off, ln, fn, sid, nf, threads, sort=True) if threads else \
        oracle_ref.build(res, off, ln, fn, sid, nf)
    assert f"kept {nf} functions\n" in stdout
    assert f"Kept {len(o['keys'])} kmers\n" in stdout
    assert f"distinct_signatures={o['distinct_signatures']}\n" in stdout
    assert f"num_seqs_with_a_signature={o['n_seqs_with_signature']}\n" in stdout
    assert _lines(os.path.join(out, "function.index")) == ref["fm"].function_index_text()
    keys, avg, fi = _parse_final_kmers(_lines(os.path.join(out, "final.kmers")))
    order = np.argsort(keys, kind="stable")
    assert np.array_equal(keys[order], o["keys"])  # every kept k-mer once (the oracle's are sorted)
    assert np.array_equal(avg[order], o["data"]["avg_from_end"])
    assert np.array_equal(fi[order], o["data"]["function_index"])
    dfl = set()
    for f in range(nf):
        if o["distinct_functions"][f]:
            dfl.add(b"%d\t%s\t%d" % (f, ref["fm"].idxf[f], o["distinct_functions"][f]))
    got = _lines(os.path.join(out, "distinct_functions")).split(b"\n")
    assert set(got[:-1]) == dfl and len(got) - 1 == len(dfl)
    # kmer_data.mph / .dat: every kept k-mer finds its record through the BDZ hash
    bdz = oracle_ref.Bdz(_lines(os.path.join(out, "kmer_data.mph")))
    assert bdz.size() == len(o["keys"])
    dat = np.frombuffer(_lines(os.path.join(out, "kmer_data.dat")), oracle_ref.STORED_DTYPE)
    idx = bdz.search(o["keys"])
    assert np.array_equal(dat[idx].view(np.uint8), o["data"].view(np.uint8))
    # recall.report.d/<fasta file name>
    fidx = _fidx(out)

    def one(item):
        path, recs = item
        return path, fr.recall_report(oracle_ref, ref["fm"], recs, fidx, o["keys"], o["data"])
    if threads:
        from concurrent.futures import ThreadPoolExecutor
        print("outputs checked; recall reports", flush=True)
        with ThreadPoolExecutor(threads) as ex:
            reports = list(ex.map(one, ref["files"][::report_stride]))
    else:
        reports = [one(x) for x in ref["files"][::report_stride]]
    for path, want in reports:
        assert _lines(os.path.join(out, "recall.report.d", os.path.basename(path))) == want, path
    return o


def _run(cmd):
    p = subprocess.run(cmd, capture_output=True, timeout=300)
    assert p.returncode == 0, p.stderr.decode()[-2000:]
    return p.stdout.decode(), p.stderr.decode()


@pytest.fixture(scope="module")
def edge_build(tmp_path_factory, gpu):
    tmp = tmp_path_factory.mktemp("cli_edge")
    d = front_data.write_edge_dirs(str(tmp / "in"))
    out = str(tmp / "kd")
    stdout, _ = _run([os.path.join(BIN, "kmers-build-signatures")] + front_data.front_args(d) + [
        "--kmer-data-dir", out, "--final-kmers", "final.kmers", "--perfect-hash", "kmer_data.mph",
        "--perfect-hash-data", "kmer_data.dat"])
    ref = fr.front([d["defs"]], [d["seqs"]], [d["keep"]], fr.read_lines(d["good_functions"]),
                   fr.read_lines(d["good_roles"]), fr.read_lines(d["deleted"]), fr.read_lines(d["ignored"]),
                   min_reps=2)
    return d, out, stdout, ref


def test_build_signatures_edge_inputs(edge_build):
    d, out, stdout, ref = edge_build
    _check_build(out, stdout, ref)
    assert os.path.getsize(os.path.join(out, "otu.index")) == 0


@pytest.fixture(scope="module")
def c1_build(tmp_path_factory, gpu):
    from signature_kmers_amd import synth
    tmp = tmp_path_factory.mktemp("cli_c1")
    info = synth.write_dirs(str(tmp / "in"), 1000, 40, per_file=100, extras=True)
    out = str(tmp / "kd")
    stdout, _ = _run([os.path.join(BIN, "kmers-build-signatures"), "-D", info["ann_dir"], "-F", info["seqs_dir"],
                      "--kmer-data-dir", out, "--final-kmers", "final.kmers", "--perfect-hash", "kmer_data.mph",
                      "--perfect-hash-data", "kmer_data.dat"])
    ref = fr.front([info["ann_dir"]], [info["seqs_dir"]])
    return info, out, stdout, ref


def test_build_signatures_c1(c1_build):
    info, out, stdout, ref = c1_build
    o = _check_build(out, stdout, ref)
    assert len(o["keys"]) > 1000
    n_rep = sum(1 for f in os.listdir(os.path.join(out, "recall.report.d")))
    assert n_rep == len(ref["files"])


def _generated_records(info, n_seqs, n_families, per_file, threads):
    """{path: [(id, b"", seq)]}: what FastaParser yields for write_dirs' files, from the generator's
    arrays (the parser itself is pinned against the reference by tests/golden/ref_fasta.npz): a
    trailing '*' alone in column 1 of a new 60-column line is dropped (fasta_parser.h:122, a bad
    id-or-data character)."""
    from signature_kmers_amd import synth
    recs = {}
    for f, (res, off, ln, _, _) in enumerate(synth.iter_file_inputs(n_seqs, n_families, per_file, workers=threads)):
        g = info["files"][f]
        rows = []
        for k in range(len(ln)):
            a, n = int(off[k]), int(ln[k])
            seq = res[a:a + n].tobytes()
            if n % 60 == 1 and seq.endswith(b"*"):
                seq = seq[:-1]
            rows.append((b"fig|%s.peg.%d" % (g.encode(), k + 1), b"", seq))
        recs[os.path.join(info["seqs_dir"], g)] = rows
    return recs


def test_build_signatures_c2(tmp_path, gpu):
    """kmers-build-signatures end to end at BASELINE configs[1] size -- 1,000,000 proteins in 250
    genome files of 4,000, 4,000 families: FASTA dirs -> function.index, final.kmers,
    distinct_functions, kmer_data.mph / .dat, recall.report.d/<file> (every 25th file's report
    byte-compared: the restatement is per-record Python) and the stdout statistics, against the
    reference restatement (oracle/front_ref.py + the oracle build and recall on all host cores).
    The run's phases (the CLI's "phases:" line) are printed (-s) for DESIGN."""
    import time
    from signature_kmers_amd import synth
    from test_gpu_scale import _threads
    n, fam = 1_000_000, 4000
    info = synth.write_dirs_parallel(str(tmp_path / "in"), n, fam, per_file=4000, workers=_threads())
    out = str(tmp_path / "kd")
    t = time.time()
    stdout, stderr = _run([os.path.join(BIN, "kmers-build-signatures"), "-D", info["ann_dir"], "-F", info["seqs_dir"],
                           "--kmer-data-dir", out, "--final-kmers", "final.kmers", "--perfect-hash", "kmer_data.mph",
                           "--perfect-hash-data", "kmer_data.dat"])
    wall = time.time() - t
    phases = [ln for ln in stderr.splitlines() if ln.startswith("phases: ")]
    print(f"\nkmers-build-signatures C2 (1M proteins): {wall:.1f} s wall\n{phases}", flush=True)
    assert len(phases) == 1
    ref = fr.front([info["ann_dir"]], [info["seqs_dir"]], records=_generated_records(info, n, fam, 4000, _threads()))
    print("reference front end done", flush=True)
    o = _check_build(out, stdout, ref, threads=_threads(), report_stride=25)  # 10 of the 250 reports
    assert len(o["keys"]) > 100_000_000 and len(ref["files"]) == 250
    assert len(os.listdir(os.path.join(out, "recall.report.d"))) == 250


def _query_dir(tmp, seed=5):
    from signature_kmers_amd import synth
    q = synth.write_dirs(str(tmp), 400, 40, per_file=100, seed=seed, extras=True, genome_base=200000)
    return q["seqs_dir"]


@pytest.mark.parametrize("ignore_hypo", [False, True])
def test_call_functions_matches_oracle(c1_build, tmp_path, ignore_hypo):
    info, out, _, _ = c1_build
    qdir = _query_dir(tmp_path / "q")
    inputs = sorted(os.path.join(qdir, f) for f in os.listdir(qdir))
    cmd = [os.path.join(BIN, "kmers-call-functions"), out] + inputs + ["-o", str(tmp_path / "calls.txt")]
    if ignore_hypo:
        cmd.append("--ignore-hypo")
    _run(cmd)
    bdz = oracle_ref.Bdz(_lines(os.path.join(out, "kmer_data.mph")))
    dat = _lines(os.path.join(out, "kmer_data.dat"))
    fidx = _fidx(out)
    want = b""
    for p in inputs:
        recs = fr.parse_fasta(_lines(p))
        w, _ = fr.call_lines(oracle_ref, recs, fidx, bdz, dat, ignore_hypo=ignore_hypo)
        want += w
    got = _lines(str(tmp_path / "calls.txt"))
    assert got == want
    assert got.count(b"\n") == sum(len(fr.parse_fasta(_lines(p))) for p in inputs)
    assert b"\tfunction " in got  # some sequences are called


def test_annotate_seqs_matches_oracle(c1_build, tmp_path):
    info, out, _, _ = c1_build
    qdir = _query_dir(tmp_path / "q", seed=9)
    calls, unc = str(tmp_path / "calls"), str(tmp_path / "uncalled")
    _run([os.path.join(BIN, "kmers-annotate-seqs"), out, str(tmp_path / "genus"), qdir, calls, unc])
    bdz = oracle_ref.Bdz(_lines(os.path.join(out, "kmer_data.mph")))
    dat = _lines(os.path.join(out, "kmer_data.dat"))
    fidx = _fidx(out)
    wc, wu = b"", b""
    for p in fr.list_files(qdir):
        c, u = fr.call_lines(oracle_ref, fr.parse_fasta(_lines(p)), fidx, bdz, dat, annotate_mode=True)
        wc += c
        wu += u
    assert _lines(calls) == wc
    assert _lines(unc) == wu


def test_matrix_distance_matches_oracle(c1_build, tmp_path):
    """kmers-matrix-distance data-dir input-file: "seq1\\tseq2\\tcount" lines (compared as a set: the
    reference prints hash order), incl. a repeated id (one SeqIdMap index) and an empty id."""
    info, out, _, _ = c1_build
    qdir = _query_dir(tmp_path / "q", seed=11)
    blob = b"".join(_lines(p) for p in fr.list_files(qdir))
    first = fr.parse_fasta(blob)[0]
    blob += b">" + first[0] + b" again\n" + first[2][5:] + b"\n>\nACDEFGHIKLMNPQ\n"
    fa = str(tmp_path / "all.faa")
    with open(fa, "wb") as fh:
        fh.write(blob)
    stdout, stderr = _run([os.path.join(BIN, "kmers-matrix-distance"), out, fa])
    recs = fr.parse_fasta(blob)
    ids = {}
    idx = np.array([ids.setdefault(r[0], len(ids)) for r in recs], np.uint32)
    names = list(ids)
    res, off, ln = fr.records_arrays(recs)
    bdz = oracle_ref.Bdz(_lines(os.path.join(out, "kmer_data.mph")))
    pairs = oracle_ref.matrix_distance(bdz, _lines(os.path.join(out, "kmer_data.dat")), res, off, ln, idx,
                                       _fidx(out).index("hypothetical protein"))
    want = {"%s\t%s\t%d" % (names[a].decode(), names[b].decode(), c) for a, b, c in pairs}
    got = stdout.split("\n")
    assert got[-1] == "" and len(got) - 1 == len(want) and set(got[:-1]) == want
    assert len(want) > 1000
    assert "kmer_hit_map size " in stderr and "write output" in stderr


def _kmer_windows(seq: bytes):
    """for_each_kmer<8> (kmer_data.h:76-102): 'X' / '*' end a run; a window is skipped when the
    next ambiguous byte lies inside it or right after it."""
    L, p, out = len(seq), 0, []

    def nxt(q):
        while q < L and seq[q] not in b"X*":
            q += 1
        return q
    na = nxt(0)
    while L >= 8 and p <= L - 8:
        if na != L and p + 8 >= na:
            p = na + 1
            na = nxt(p)
            continue
        out.append(p)
        p += 1
    return out


@pytest.mark.parametrize("ignore_hypo", [False, True])
def test_call_functions_debug_hits(c1_build, tmp_path, ignore_hypo):
    """--debug-hits prints the reference's hit_cb line per DB hit (kmers-call-functions.cc:109-118:
    kmer, offset, function, median, mean, var, sqrt(var)), after the hypothetical filter
    (call_functions.tcc:284-291), before each file's calls; the calls file is unchanged."""
    info, out, _, _ = c1_build
    qdir = _query_dir(tmp_path / "q", seed=13)
    inputs = sorted(os.path.join(qdir, f) for f in os.listdir(qdir))[:2]
    cmd = [os.path.join(BIN, "kmers-call-functions"), out] + inputs + ["-o", str(tmp_path / "calls.txt"),
                                                                        "--debug-hits"]
    if ignore_hypo:
        cmd.append("--ignore-hypo")
    stdout, _ = _run(cmd)
    bdz = oracle_ref.Bdz(_lines(os.path.join(out, "kmer_data.mph")))
    dat = np.frombuffer(_lines(os.path.join(out, "kmer_data.dat")), oracle_ref.STORED_DTYPE)
    fidx = _fidx(out)
    hypo = fidx.index("hypothetical protein")
    want, calls_want = [], b""
    for p in inputs:
        recs = fr.parse_fasta(_lines(p))
        for _, _, seq in recs:
            pos = _kmer_windows(seq)
            if not pos:
                continue
            keys = np.array([int.from_bytes(seq[q:q + 8], "little") for q in pos], np.uint64)
            idx = bdz.search(keys)
            for q, k, ix in zip(pos, keys, idx):
                if ix >= len(dat):
                    continue
                d = dat[ix]
                if ignore_hypo and int(d["function_index"]) == hypo:
                    continue
                fn = fidx[d["function_index"]] if d["function_index"] < len(fidx) else ""
                want.append("%s\t%d\t%s\t%d\t%d\t%d\t%s\t" % (int(k).to_bytes(8, "little").decode("latin-1"), q, fn,
                                                             d["median"], d["mean"], d["var"],
                                                             fr.fmt_g(float(np.sqrt(float(d["var"]))))))
        w, _ = fr.call_lines(oracle_ref, recs, fidx, bdz, _lines(os.path.join(out, "kmer_data.dat")),
                             ignore_hypo=ignore_hypo)
        calls_want += w
    got = stdout.split("\n")
    assert got[-1] == "" and got[:-1] == want
    assert len(want) > 1000
    assert _lines(str(tmp_path / "calls.txt")) == calls_want


def test_call_functions_boost_math_legacy(c1_build, tmp_path):
    """--boost-math-stats legacy: the calls of a reference compiled against the older Boost.Math
    (single running mean, MAD = |x(mid)|; call_functions.tcc:51-53) -- the oracle's modes 1/1."""
    info, out, _, _ = c1_build
    qdir = _query_dir(tmp_path / "q", seed=17)
    inputs = sorted(os.path.join(qdir, f) for f in os.listdir(qdir))
    _run([os.path.join(BIN, "kmers-call-functions"), out] + inputs + ["-o", str(tmp_path / "calls.txt"),
                                                                      "--boost-math-stats", "legacy"])
    bdz = oracle_ref.Bdz(_lines(os.path.join(out, "kmer_data.mph")))
    dat = _lines(os.path.join(out, "kmer_data.dat"))
    fidx = _fidx(out)
    hypo = fidx.index("hypothetical protein")
    want = b""
    for p in inputs:
        recs = fr.parse_fasta(_lines(p))
        res, off, ln = fr.records_arrays(recs)
        coff, calls = oracle_ref.annotate(bdz, dat, res, off, ln, hypo_index=hypo, mean_mode=1, mad_mode=1)
        for r, (pid, _, _) in enumerate(recs):
            fi, func, score, _ = oracle_ref.find_best_call(calls[coff[r]:coff[r + 1]], fidx)
            want += b"%s\t%s\t%d\t%s\n" % (pid, func.encode("latin-1"), fi, fr.fmt_g(score).encode())
    assert _lines(str(tmp_path / "calls.txt")) == want
    p = subprocess.run([os.path.join(BIN, "kmers-call-functions"), out, inputs[0], "--boost-math-stats", "old"],
                       capture_output=True, timeout=120)
    assert p.returncode != 0 and b"--boost-math-stats" in p.stderr


def test_matrix_distance_row_bands_multi_rank(c1_build, tmp_path):
    """kmers-matrix-distance --n-gpus 2/3 --comm host (--same-device: every rank on the one GPU):
    rank r looks up its range of the records, hits go to their k-mer's owner and k-mer groups to
    the row bands (skm_matrix_tile_rows) over the ranks' socketpairs, rank r counts its band and
    rank 0 prints the bands in rank order -- byte-identical to the one-process output."""
    info, out, _, _ = c1_build
    qdir = _query_dir(tmp_path / "q", seed=19)
    fa = str(tmp_path / "all.faa")
    with open(fa, "wb") as fh:
        fh.write(b"".join(_lines(p) for p in fr.list_files(qdir)))
    one, err1 = _run([os.path.join(BIN, "kmers-matrix-distance"), out, fa])
    assert one.count("\n") > 1000
    size1 = [ln for ln in err1.splitlines() if ln.startswith("kmer_hit_map size ")]
    for n, comm in ((2, ["--comm", "host"]), (3, [])):  # --same-device defaults to the host transport
        many, err = _run([os.path.join(BIN, "kmers-matrix-distance"), out, fa, "--n-gpus", str(n), "--same-device"]
                         + comm)
        assert many == one, n
        # the map's size summed over the owners: the one-process line
        assert [ln for ln in err.splitlines() if ln.startswith("kmer_hit_map size ")] == size1, (n, err)


def test_build_signatures_multi_rank_host_comm(tmp_path, gpu):
    """kmers-build-signatures --n-gpus 2 --comm host: two forked ranks on the one GPU, each
    building its contiguous range of files and exchanging occurrences by owner through the
    socketpair host transport; rank 0 writes every output -- the same files and stdout lines
    as one process."""
    from signature_kmers_amd import synth
    info = synth.write_dirs(str(tmp_path / "in"), 1000, 40, per_file=100, extras=True)
    outs = {}
    for tag, extra in (("one", []), ("two", ["--n-gpus", "2", "--comm", "host"])):
        o = str(tmp_path / tag)
        stdout, _ = _run([os.path.join(BIN, "kmers-build-signatures"), "-D", info["ann_dir"], "-F", info["seqs_dir"],
                          "--kmer-data-dir", o, "--final-kmers", "final.kmers", "--perfect-hash", "kmer_data.mph",
                          "--perfect-hash-data", "kmer_data.dat"] + extra)
        outs[tag] = (o, stdout)
    (o1, s1), (o2, s2) = outs["one"], outs["two"]
    assert s1 == s2
    for name in ("final.kmers", "distinct_functions", "function.index", "kmer_data.dat"):
        assert sorted(_lines(os.path.join(o1, name)).split(b"\n")) == sorted(_lines(os.path.join(o2, name)).split(b"\n")), name
    for f in os.listdir(os.path.join(o1, "recall.report.d")):
        assert _lines(os.path.join(o1, "recall.report.d", f)) == _lines(os.path.join(o2, "recall.report.d", f)), f


def test_build_signatures_rank_failure_stops_the_job(tmp_path, gpu):
    """--n-gpus 2 --comm rccl with rank 1 failing before it joins the communicator: rank 0 would
    block in the RCCL init forever; its child watcher terminates the job with exit status 1
    (on a one-GPU box rank 1 also fails earlier, on device 1 -- the same path)."""
    from signature_kmers_amd import synth
    info = synth.write_dirs(str(tmp_path / "in"), 200, 10, per_file=100, extras=False)
    env = dict(os.environ, SKM_CLI_FAIL_RANK="1")
    p = subprocess.run([os.path.join(BIN, "kmers-build-signatures"), "-D", info["ann_dir"], "-F", info["seqs_dir"],
                        "--kmer-data-dir", str(tmp_path / "o"), "--n-gpus", "2", "--comm", "rccl"],
                       capture_output=True, timeout=120, env=env)
    err = p.stderr.decode()
    assert p.returncode == 1, err[-2000:]
    assert "rank 1 failed" in err, err[-2000:]
