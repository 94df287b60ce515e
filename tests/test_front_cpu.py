"""CPU tests of the CLI host front end (no GPU): FASTA parsing, SEED assignment rules, function
selection, function.index and the build input of bin/kmers-build-signatures, checked against the
independent Python restatement in oracle/front_ref.py."""
import os
import subprocess

import numpy as np
import pytest

import front_data
from conftest import ROOT

import oracle.front_ref as fr  # noqa: E402  (test infrastructure)

BIN = os.path.join(ROOT, "bin")


@pytest.fixture(scope="module")
def tools(skm):
    for t in ("kmers-build-signatures", "kmers-call-functions", "kmers-annotate-seqs", "skm-front-probe"):
        if not os.path.exists(os.path.join(BIN, t)):
            subprocess.check_call(["make", "-C", ROOT, "-j8", "tools"])
            break
    return BIN


def _probe(tools, strings):
    inp = "\n".join(s.hex() if s else "-" for s in strings) + "\n"
    out = subprocess.run([os.path.join(tools, "skm-front-probe")], input=inp.encode(), capture_output=True,
                         check=True).stdout.decode().splitlines()
    un = lambda h: b"" if h == "-" else bytes.fromhex(h)  # noqa: E731
    res = []
    for line in out:
        c = line.split("\t")
        roles = un(c[6]).split(b"\x01") if int(c[5]) else []
        res.append(dict(split=(un(c[0]), un(c[1]), un(c[2])), trunc=c[3] == "1", strip=un(c[4]), roles=roles,
                        genome=(un(c[8]), un(c[9])) if c[7] == "1" else None,
                        fig=un(c[11]) if c[10] == "1" else None))
    return res


HANDPICKED = [
    b"", b"alpha", b"alpha # comment", b"alpha  ## fragment x", b"alpha #no-space", b"alpha# x", b"#x y",
    b" # lead", b"a # b # c", b"a\t#\tb", b"a #", b"a # ", b"frag", b"missing part", b"x\nfrag",
    b"beta / gamma", b"beta/gamma", b"beta @ gamma", b"a; b", b"a ;b", b"a ; b ; c", b" / a", b"a / ", b"; a",
    b"a /  @ b", b"a # c / d", b" f [g]", b"  [g]", b" [g]", b"\tf x [Gen sp]", b" f [g]x", b" f [a]b]",
    b" f [a[b]", b" f[g]", b" f  [g h]", b" a [b] [c]", b" f []", b"fig|123.4.peg.5", b"xfig|1.2",
    b"fig|1.", b"fig|.2 fig|3.4", b"fig|12a.3",
]


def test_regex_matchers_match_python_re(tools):
    rng = np.random.default_rng(3)
    alphabet = list(b"ab #/@;[] \tfrgmistunc|.0123\n")
    rand = [bytes(rng.choice(alphabet, size=int(rng.integers(0, 24))).astype(np.uint8)) for _ in range(3000)]
    strings = HANDPICKED + rand
    got = _probe(tools, strings)
    assert len(got) == len(strings)
    for s, g in zip(strings, got):
        assert g["split"] == fr.split_func_comment(s), s
        assert g["trunc"] == fr.is_truncated_comment(s), s
        assert g["strip"] == fr.strip_func_comment(s), s
        assert g["roles"] == fr.roles_of_function(s), s
        assert g["genome"] == fr.match_genome(s), s
        m = fr.RE_FIGID.search(s)
        assert g["fig"] == (m.group(1) if m else None), s


def test_fasta_parser_edge_cases():
    data = b"junk\n>id1 def one\r\nACGT\n*MK\nmk1-*\n\n>\nAAAA\n>id2\tx\n>id3\nQQ"
    recs = fr.parse_fasta(data)
    # '*' opening a continuation line, '1' and '-' are dropped; a header right after a header
    # line is read as (bad) sequence data in s_data, so "id3" becomes residues of id2
    assert recs == [(b"id1", b" def one", b"ACGTMKmk*"), (b"id2", b"\tx", b"idQQ")]


def test_fasta_headers_only_parse_matches_full(tools, tmp_path):
    # the headers-only parse (other ranks' files in the multi-rank CLI) yields the same records,
    # offsets and lengths as the full parse, and parses the same (bad) characters the same way
    data = (b"junk\n>id1 def one\r\nACGT\n*MK\nmk1-*\n\n>\nAAAA\n>id2\tx\n>id3\nQQ\n"
            + b"".join(b">s%d fn %d\n%s\n" % (i, i, b"ACDEFGHIKLMNPQRSTVWY"[: 1 + i % 20] * (1 + i % 7)) for i in range(300)))
    f = tmp_path / "x.faa"
    f.write_bytes(data)
    probe = os.path.join(tools, "skm-front-probe")
    full = subprocess.run([probe, "--fasta", str(f), "1"], capture_output=True, check=True)
    light = subprocess.run([probe, "--fasta", str(f), "0"], capture_output=True, check=True)
    fl, ll = full.stdout.decode().splitlines(), light.stdout.decode().splitlines()
    assert fl[:-1] == ll[:-1] and len(fl) == 303
    nf, nl = fl[-1].split(), ll[-1].split()
    assert nf[1] == nl[1] == nf[3] and nl[3] == "0"
    assert full.stderr == light.stderr and b"Bad data character" in full.stderr


def _run_front(tools, d, out, extra=()):
    cmd = [os.path.join(tools, "kmers-build-signatures")] + front_data.front_args(d) + [
        "--kmer-data-dir", out, "--dump-extract", os.path.join(out, "extract.bin")] + list(extra)
    p = subprocess.run(cmd, capture_output=True, check=True)
    return p.stdout.decode(), p.stderr.decode()


def test_front_end_matches_restatement(tools, tmp_path):
    d = front_data.write_edge_dirs(str(tmp_path / "in"))
    out = str(tmp_path / "out")
    stdout, _ = _run_front(tools, d, out)
    ref = fr.front([d["defs"]], [d["seqs"]], [d["keep"]], fr.read_lines(d["good_functions"]),
                   fr.read_lines(d["good_roles"]), fr.read_lines(d["deleted"]), fr.read_lines(d["ignored"]),
                   min_reps=2)
    assert f"kept {ref['n_kept_functions']} functions" in stdout
    with open(os.path.join(out, "function.index"), "rb") as fh:
        assert fh.read() == ref["fm"].function_index_text()
    got = fr.read_dump(os.path.join(out, "extract.bin"))
    for g, r, name in zip(got, ref["build"], ["residues", "off", "len", "func", "seq_id"]):
        assert np.array_equal(g, r), name
    assert os.path.getsize(os.path.join(out, "otu.index")) == 0
    with open(os.path.join(out, "genomes"), "rb") as fh:
        assert fh.read() == b"empty genomes\n"
    # the edge data exercises the rules it is meant to
    names = set(ref["fm"].fidx)
    assert b"iota rare" in names and b"lambda ignored" not in names and b"hypothetical protein" in names
    assert b"zeta transporter @ eta permease" in names
    assert len(got[0]) > 0 and (got[3] != 0xFFFF).all()


def test_front_end_synthetic_layout_matches_generator(tools, tmp_path):
    from signature_kmers_amd import synth
    info = synth.write_dirs(str(tmp_path / "in"), 1000, 40, per_file=100, extras=True)
    out = str(tmp_path / "out")
    subprocess.run([os.path.join(tools, "kmers-build-signatures"), "-D", info["ann_dir"], "-F", info["seqs_dir"],
                    "--kmer-data-dir", out, "--min-reps-required", "1", "--dump-extract",
                    os.path.join(out, "x.bin")], capture_output=True, check=True)
    res, off, ln, fn, sid = fr.read_dump(os.path.join(out, "x.bin"))
    ref = fr.front([info["ann_dir"]], [info["seqs_dir"]], min_reps=1)
    for g, r in zip((res, off, ln, fn, sid), ref["build"]):
        assert np.array_equal(g, r)
    # FastaParser drops a '*' that opens a continuation line (fasta_parser.h:122): the generator's
    # trailing '*' is lost exactly when it lands in column 1 of a new 60-column line
    p = info["proteome"]
    last = p.residues[(p.seq_off + p.seq_len - 1).astype(np.int64)]
    lost = int(((p.seq_len % 60 == 1) & (last == ord("*"))).sum())
    assert int(ln.astype(np.int64).sum()) == int(p.seq_len.astype(np.int64).sum()) - lost


def test_definition_bad_lines_reported_in_order(tools, tmp_path):
    """load_id_assignments (function_map.h:62-104) parses the definition files on host threads:
    lines without a tab -- an empty line and a last line without a newline included -- are reported
    as "bad line N" with getline's numbering, in line order within a file (the files in directory
    listing order, as before), and the assignments of the good lines still apply."""
    defs = tmp_path / "defs"
    seqs = tmp_path / "seqs"
    defs.mkdir()
    seqs.mkdir()
    (defs / "a").write_bytes(b"fig|1.1.peg.1\talpha protein\nnotab line\n\nfig|1.1.peg.2\tbeta protein # note\nlast")
    (defs / "b").write_bytes(b"fig|1.1.peg.3\tgamma protein\n\n")
    (seqs / "1.1").write_bytes(b">fig|1.1.peg.1\nMKVLAAGIVGLLLAWQ\n>fig|1.1.peg.2\nMKTAYIAKQRQISFVK\n"
                               b">fig|1.1.peg.3\nMSTNPKPQRKTKRNTNRR\n")
    out = tmp_path / "out"
    cmd = [os.path.join(tools, "kmers-build-signatures"), "-D", str(defs), "-F", str(seqs), "--kmer-data-dir", str(out),
           "--min-reps-required", "1", "--dump-extract", str(out / "extract.bin")]
    p = subprocess.run(cmd, capture_output=True, check=True)
    bad = [ln for ln in p.stderr.decode().splitlines() if ln.startswith("bad line")]
    in_a = [ln for ln in bad if ln.endswith(f'"{defs / "a"}"')]
    assert in_a == [f'bad line 2 in file "{defs / "a"}"', f'bad line 3 in file "{defs / "a"}"',
                    f'bad line 5 in file "{defs / "a"}"']
    assert [ln for ln in bad if ln not in in_a] == [f'bad line 2 in file "{defs / "b"}"']
    names = {ln.split(b"\t")[1] for ln in (out / "function.index").read_bytes().splitlines()}
    assert {b"alpha protein", b"beta protein", b"gamma protein"} <= names
