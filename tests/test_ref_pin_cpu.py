"""CPU tests against golden vectors produced by the REFERENCE ITSELF (no GPU).

tests/golden/ref_windows.npz and ref_fasta.npz hold the outputs of the reference's own
for_each_kmer<8> (kmer_data.h:76-102) and FastaParser (fasta_parser.h:38-144,
fasta_parser.cc:17-36), compiled unchanged from /root/reference by oracle/Makefile.ref and driven
over adversarial inputs by tests/golden/make_golden_ref.py (oracle/ref_pin.cpp).  They pin:
  - the oracle's window iterator (oracle_kmer_windows), which every annotate / matrix / recall
    parity test relies on;
  - the oracle's FASTA restatement (oracle/front_ref.py parse_fasta);
  - the product's host FASTA parser (csrc/front/skm_front.cpp via bin/skm-front-probe), records
    and error reports both.
The device window iterator is checked against the same vectors in test_gpu_annotate.py."""
import os
import subprocess

import numpy as np
import pytest

import oracle_ref
from conftest import ROOT

import oracle.front_ref as fr  # noqa: E402  (test infrastructure)

GOLD = os.path.join(ROOT, "tests", "golden")


def _split(flat, off):
    return [bytes(flat[off[i]:off[i + 1]]) for i in range(len(off) - 1)]


def ref_windows():
    z = np.load(os.path.join(GOLD, "ref_windows.npz"))
    seqs = _split(z["seqs"], z["seq_off"])
    wins = [z["win"][z["win_off"][i]:z["win_off"][i + 1]] for i in range(len(seqs))]
    return seqs, wins


def _parse_lines(text: bytes):
    """ref_pin / skm-front-probe --fasta-hex lines -> (records [(id, def, seq)], errors
    [(line, message, id)])."""
    un = lambda h: b"" if h == "-" else bytes.fromhex(h)  # noqa: E731
    recs, errs = [], []
    for ln in text.decode().splitlines():
        c = ln.split(" ")
        if c[0] == "R":
            recs.append((un(c[1]), un(c[2]), un(c[3])))
        elif c[0] == "E":
            errs.append((int(c[1]), un(c[2]), un(c[3])))
        else:
            raise AssertionError(ln)
    return recs, errs


def ref_fasta():
    z = np.load(os.path.join(GOLD, "ref_fasta.npz"))
    blobs = _split(z["blobs"], z["blob_off"])
    full = [_parse_lines(t) for t in _split(z["out"], z["out_off"])]
    simple = [_parse_lines(t) for t in _split(z["sout"], z["sout_off"])]
    return blobs, full, simple


def test_golden_vectors_cover_the_adversarial_cases():
    seqs, wins = ref_windows()
    assert len(seqs) > 1500 and sum(len(w) for w in wins) > 20000
    assert any(len(s) < 8 for s in seqs) and any(s.endswith(b"X") for s in seqs) and any(b"x" in s for s in seqs)
    blobs, full, _ = ref_fasta()
    errs = [e for _, es in full for e in es]
    assert {m for _, m, _ in errs} >= {b"Missing >"}
    assert any(m.startswith(b"Bad data character") for _, m, _ in errs)
    assert any(m.startswith(b"Bad id or data character") for _, m, _ in errs)
    # the second parse_complete of the callers (signature_build.tcc:100-101) fires one more
    # callback, always with an empty id -- which every caller skips
    assert all(recs and recs[-1] == (b"", b"", b"") for recs, _ in full)


def test_oracle_window_iterator_matches_reference():
    seqs, wins = ref_windows()
    for s, w in zip(seqs, wins):
        got = oracle_ref.kmer_windows(s)
        assert np.array_equal(got, w.astype(np.uint32)), s


def test_front_ref_parse_matches_reference():
    blobs, full, simple = ref_fasta()
    for b, (recs, _), (srecs, _) in zip(blobs, full, simple):
        want = [r for r in recs if r[0]]  # callers skip empty ids (signature_build.tcc:124)
        assert fr.parse_fasta(b) == want, b
        # the (id, seq) callback form sees the same records
        assert [(i, s) for i, _, s in srecs if i] == [(i, s) for i, _, s in want], b


@pytest.fixture(scope="module")
def probe(skm):
    p = os.path.join(ROOT, "bin", "skm-front-probe")
    if not os.path.exists(p):
        subprocess.check_call(["make", "-C", ROOT, "-j8", "tools"])
    return p


def test_product_fasta_parser_matches_reference(probe):
    blobs, full, _ = ref_fasta()
    inp = "".join((b.hex() if b else "-") + "\n" for b in blobs).encode()
    out = subprocess.run([probe, "--fasta-hex"], input=inp, capture_output=True, check=True).stdout
    per = out.split(b"END\n")
    assert len(per) == len(blobs) + 1 and per[-1] == b""
    for b, text, (recs, errs) in zip(blobs, per[:-1], full):
        grecs, gerrs = _parse_lines(text)
        assert grecs == [r for r in recs if r[0]], b
        # the same error reports (message, line number, current id), in order
        assert gerrs == errs, b


# ------------------------------------------------------------------ split / record layout
# tests/golden/ref_split.npz: the reference's own split() (operators.h:80-91) over adversarial
# strings and its StoredKmerData / KmerAttributes layout (kmer_data.h:105-128), from oracle/_ref.
def ref_split():
    z = np.load(os.path.join(GOLD, "ref_split.npz"))
    strs, delims = _split(z["strs"], z["str_off"]), _split(z["delims"], z["delim_off"])
    flat = _split(z["parts"], z["part_off"])
    parts, k = [], 0
    for n in z["nparts"]:
        parts.append(flat[k:k + int(n)])
        k += int(n)
    return list(zip(strs, delims, parts)), [int(x) for x in z["layout"]]


def test_split_vectors_cover_the_edge_cases():
    cases, _ = ref_split()
    got = {(s, d): p for s, d, p in cases}
    assert got[(b"", b" / ")] == [b""]                      # empty string: one empty field
    assert got[(b"a / ", b" / ")] == [b"a", b""]            # trailing delimiter: trailing empty field
    assert got[(b" / a", b" / ")] == [b"", b"a"]
    assert got[(b"a / / b", b" / ")] == [b"a", b"/ b"]      # the delimiter is a whole string
    assert got[(b"12\t\t", b"\t")] == [b"12", b"", b""]
    assert len(cases) > 400


def test_oracle_split_matches_reference():
    cases, _ = ref_split()
    for s, d, p in cases:
        assert oracle_ref.split(s, d) == p, (s, d)


def test_product_split_matches_reference(probe):
    cases, _ = ref_split()
    inp = "".join(f"{s.hex() or '-'} {d.hex() or '-'}\n" for s, d, _ in cases).encode()
    out = subprocess.run([probe, "--split"], input=inp, capture_output=True, check=True).stdout.decode().splitlines()
    assert len(out) == len(cases)
    for ln, (s, d, p) in zip(out, cases):
        c = ln.split(" ")
        assert c[0] == "P" and int(c[1]) == len(p), (s, d, ln)
        assert [b"" if h == "-" else bytes.fromhex(h) for h in c[2:]] == p, (s, d)


def test_product_read_function_index_matches_reference_split(probe, tmp_path):
    """read_function_index (call_functions.tcc:123-148) restated from the pinned split: slot
    stoi(parts[0]) = parts[1] of split(line, "\\t"), max id + 1 slots, later lines win."""
    cases, _ = ref_split()
    rng = np.random.default_rng(5)
    names = [p[1] for s, d, p in cases if d == b"\t" and len(p) > 1] + \
            [b"a / b", b"", b"x / ", b"name with / slash", b"  padded  "]
    lines, want = [], {}
    for k, nm in enumerate(names):
        idx = int(rng.integers(0, 60)) if k % 3 else k
        extra = b"\t".join(bytes(rng.choice(list(b"0123 /"), size=int(rng.integers(0, 4))).astype(np.uint8))
                           for _ in range(int(rng.integers(0, 4))))
        line = str(idx).encode() + b"\t" + nm + (b"\t" + extra if extra or k % 2 else b"")
        lines.append(line)
        parts = oracle_ref.split(line, b"\t")   # == the reference's split (test above)
        want[int(parts[0])] = parts[1]
    f = tmp_path / "function.index"
    f.write_bytes(b"\n".join(lines) + b"\n")
    out = subprocess.run([probe, "--function-index", str(f)], capture_output=True, check=True).stdout.decode()
    got = [ln.split(" ") for ln in out.splitlines()]
    assert len(got) == max(want) + 1
    for i, h in got:
        assert (b"" if h == "-" else bytes.fromhex(h)) == want.get(int(i), b""), i


def test_stored_kmer_data_layout_matches_reference(tmp_path):
    """skm_stored_kmer_data (include/skm.h), the Python mirror STORED_DTYPE and the oracle's
    record all have the reference's StoredKmerData layout: the 10-byte kmer_data.dat record."""
    import signature_kmers_amd as skm_pkg
    _, lay = ref_split()
    size, align, offs = lay[0], lay[1], lay[2:7]
    assert (size, offs) == (10, [0, 2, 4, 6, 8])
    for dt in (skm_pkg.STORED_DTYPE, oracle_ref.STORED_DTYPE):
        assert dt.itemsize == size
        assert [dt.fields[n][1] for n in ("avg_from_end", "function_index", "mean", "median", "var")] == offs
    src = tmp_path / "lay.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "skm.h"\nint main(void) {\n'
                   '  printf("%zu %zu %zu %zu %zu %zu %zu\\n", sizeof(skm_stored_kmer_data), _Alignof(skm_stored_kmer_data),\n'
                   '    offsetof(skm_stored_kmer_data, avg_from_end), offsetof(skm_stored_kmer_data, function_index),\n'
                   '    offsetof(skm_stored_kmer_data, mean), offsetof(skm_stored_kmer_data, median),\n'
                   '    offsetof(skm_stored_kmer_data, var));\n  return 0;\n}\n')
    exe = tmp_path / "lay"
    subprocess.check_call(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)])
    got = [int(x) for x in subprocess.check_output([str(exe)]).split()]
    assert got == [size, align] + offs
    # KmerAttributes (kmer_data.h:105-112) is the reference's in-memory build record; the build
    # keeps its fields in the 16-byte element instead -- pinned for the record
    assert lay[7:] == [16, 4, 0, 2, 4, 8, 12]
