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
