#!/usr/bin/env python3
"""Golden vectors from the REFERENCE ITSELF (TEST INFRASTRUCTURE).

The parts of olsonanl/signature_kmers that compile here unchanged -- for_each_kmer<8>
(kmer_data.h:76-102) and FastaParser (fasta_parser.h:38-144, fasta_parser.cc:17-36) -- are built
from /root/reference by oracle/Makefile.ref into oracle/_ref/ref_pin (oracle/ref_pin.cpp drives
them).  This script feeds them adversarial inputs and stores inputs + the reference's outputs:

ref_windows.npz  seqs (concatenated bytes) / seq_off [n+1]; win (concatenated offsets) / win_off
                 [n+1] = for_each_kmer<8>'s offsets per sequence.  The sequences put 'X' / '*'
                 at every offset of a window and at the sequence end, pairs of them, runs, lower
                 case 'x' (not ambiguous), B / Z / U / O / J, lengths 0..40, and long random ones.
ref_split.npz    split(s, delim) of operators.h:80-91 over adversarial strings: strs / str_off,
                 delims / delim_off, parts / part_off (the parts of all cases concatenated) and
                 nparts [n] (parts per case); plus `layout` = sizeof, alignof and offsetof of
                 StoredKmerData (avg_from_end, function_index, mean, median, var) and of
                 KmerAttributes (func_index, otu_index, offset, seq_id, protein_length),
                 kmer_data.h:105-128, as the reference compiles them.
ref_fasta.npz    blobs / blob_off [n+1] (FASTA file images); out / out_off [n+1] = ref_pin's
                 lines per blob for the load_kmers_from_fasta driving ("F": def callback, parse,
                 then the caller's second parse_complete) and sout / sout_off for the (id, seq)
                 callback driving of function_map.h / call_functions.tcc ("S").  Blobs hold
                 '\\r', a leading '*' on a continuation line, bad characters (digits, '-', '#',
                 bytes >= 0x80), empty ids, headers without data, text before the first '>',
                 no final newline, and random mixtures of those.

usage: python tests/golden/make_golden_ref.py   (needs /root/reference; writes next to this script)
"""
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF_PIN = os.path.join(ROOT, "oracle", "_ref", "ref_pin")

AA = b"ACDEFGHIKLMNPQRSTVWY"


def window_inputs(rng):
    seqs = []
    # one ambiguous byte at every offset, lengths 0..24
    for L in range(0, 25):
        base = bytes(rng.choice(list(AA), size=L).astype(np.uint8)) if L else b""
        seqs.append(base)
        for p in range(L):
            for a in b"X*x":
                s = bytearray(base)
                s[p] = a
                seqs.append(bytes(s))
    # two ambiguous bytes at every pair of offsets, lengths 9..20
    for L in (9, 12, 16, 17, 20):
        base = bytearray(rng.choice(list(AA), size=L).astype(np.uint8))
        for p in range(L):
            for q in range(p + 1, L):
                s = bytearray(base)
                s[p] = ord("X")
                s[q] = ord("*")
                seqs.append(bytes(s))
    # runs, all-ambiguous, unusual letters
    for s in (b"XXXXXXXXXXXX", b"********", b"ACDEFGHIX", b"XACDEFGHI", b"ACDEFGH*", b"*ACDEFGH",
              b"ACDEFGHIK*", b"ACDEFGHIKX", b"AAAAAAAAXXAAAAAAAA", b"AAAAAAAA*AAAAAAAA*AAAAAAAA",
              b"BZUOJBZUOJBZUOJ", b"acdefghiklmnpqrs", b"ACDEFGHIkx*lmnpqrstvwy", b"ACDEFGHI" * 5):
        seqs.append(s)
    # long random sequences with sparse ambiguity
    letters = np.frombuffer(AA + b"acdBZUXX**", np.uint8)
    for _ in range(300):
        L = int(rng.integers(0, 400))
        seqs.append(bytes(rng.choice(letters, size=L, p=None).astype(np.uint8)))
    return seqs


def fasta_inputs(rng):
    blobs = [
        b"",
        b">",
        b">id",
        b">id\n",
        b">id\nACDEFGHIK",
        b">id def\nACDEFGHIK\n",
        b">id\tdef two\r\nACDE\r\nFGHI\r\n",
        b">id1 d\nACGT\n*MK\nmk1-*\n\n>\nAAAA\n>id2\tx\n>id3\nQQ",
        b"junk\n>id1\nAAAA\n",
        b"\n\n>a\nAA\n\n\n>b\nBB\n",
        b">a\n*AAA\n",
        b">a\nAAA*\n*BBB\nC*C\n",
        b">a\n>b\nCC\n",
        b"> lead space\nAC\n",
        b">a b c\nAC DE\n",
        b">a\nAC\xc3\xa9DE\n>\xc3\xa9id\nKK\n",
        b">a\nAC\nD1E\n-F\n#G\n>b\n",
        b">a\r\n\r\nAC\r\n>b\r\nDE",
        b">x\n" + b"ACDEFGHIKLMNPQRSTVWY" * 30 + b"\n",
        b">only header 1\n>only header 2\n",
        b">a\n\n\n\nA\n",
    ]
    alphabet = list(b">>>\n\n\n\r \tACdeXx**1-#") + [0xC3, 0x7F, 0x00]
    for _ in range(1500):
        L = int(rng.integers(0, 48))
        blobs.append(bytes(rng.choice(alphabet, size=L).astype(np.uint8)))
    # structured random files: records with random ids, defs, wrapped residues and noise
    for _ in range(300):
        out = bytearray()
        if rng.random() < 0.2:
            out += b"noise\n"
        for _r in range(int(rng.integers(0, 6))):
            out += b">" + bytes(rng.choice(list(b"abc|.0123_"), size=int(rng.integers(0, 6))).astype(np.uint8))
            if rng.random() < 0.5:
                out += b" " + bytes(rng.choice(list(b"def ghi\t#"), size=int(rng.integers(0, 8))).astype(np.uint8))
            out += b"\r\n" if rng.random() < 0.2 else b"\n"
            for _l in range(int(rng.integers(0, 4))):
                line = bytearray(rng.choice(list(b"ACDEFGHIKLMNXx*"), size=int(rng.integers(0, 12))).astype(np.uint8))
                if line and rng.random() < 0.15:
                    line[int(rng.integers(0, len(line)))] = int(rng.choice(list(b"1-# \x80")))
                out += line + b"\n"
        if out and rng.random() < 0.3:
            out = out[:-1]
        blobs.append(bytes(out))
    return blobs


def split_inputs(rng):
    """(s, delim) cases: the two delimiters the path splits on -- " / " (find_best_call's fusion
    parts, call_functions.tcc:487) and "\\t" (read_function_index, :143) -- over empty fields,
    leading / trailing / doubled delimiters, near-miss delimiters and names containing '/'."""
    fixed = [b"", b" / ", b"a / ", b" / a", b"a / / b", b"a /  / b", b"a / b / c", b"a  /  b", b"a/b", b"a /b",
             b"a/ b", b" /  / ", b"a / b / ", b" / / ", b"/", b"//", b" /", b"/ ", b"a / b/c / d", b"and/or / x",
             b"1,3-beta / 1,4-alpha / ", b"x // y", b"a  / b", b"a /\tb", b"function 00001 / function 00003"]
    cases = [(s, b" / ") for s in fixed]
    tabs = [b"", b"\t", b"a\t", b"\ta", b"a\t\tb", b"0\talpha\t3\t1\t1\t0\t0", b"2\tgamma / delta\t9",
            b"12\t\t", b"7\tx\ty\tz\t", b"\t\t\t", b"5\tname with / slash\t1", b"a b\tc d"]
    cases += [(s, b"\t") for s in tabs]
    alphabet = list(b"ab /\t")
    for _ in range(400):
        L = int(rng.integers(0, 24))
        s = bytes(rng.choice(alphabet, size=L).astype(np.uint8))
        cases.append((s, b" / " if rng.random() < 0.6 else b"\t"))
    cases += [(b"a--b----c--", b"--"), (b"xyz", b"xyz"), (b"xyzxyz", b"xyz"), (b"aaa", b"aa")]
    return cases


def hexs(b: bytes) -> str:
    return b.hex() if b else "-"


def run(reqs):
    return run_lines("".join(f"{op} {hexs(b)}\n" for op, b in reqs))


def run_lines(inp: str):
    return subprocess.run([REF_PIN], input=inp.encode(), capture_output=True, check=True).stdout


def cat(items, dtype=np.uint8):
    off = np.zeros(len(items) + 1, np.int64)
    off[1:] = np.cumsum([len(x) for x in items])
    flat = np.concatenate([np.frombuffer(x, np.uint8) if dtype == np.uint8 else np.asarray(x, dtype)
                           for x in items]) if items else np.zeros(0, dtype)
    return flat.astype(dtype), off


def main():
    subprocess.check_call(["make", "-s", "-C", ROOT, "-f", "oracle/Makefile.ref"])
    rng = np.random.default_rng(20241115)
    seqs = window_inputs(rng)
    lines = run([("W", s) for s in seqs]).decode().splitlines()
    assert len(lines) == len(seqs)
    wins = []
    for ln in lines:
        body = ln[2:]
        wins.append(np.array([int(x) for x in body.split(",")] if body != "-" else [], np.int32))
    s_flat, s_off = cat(seqs)
    w_flat, w_off = cat(wins, np.int32)
    np.savez_compressed(os.path.join(HERE, "ref_windows.npz"), seqs=s_flat, seq_off=s_off, win=w_flat, win_off=w_off)

    cases = split_inputs(np.random.default_rng(20261018))  # own stream: ref_fasta stays as it was
    text = run_lines("".join(f"P {hexs(a)} {hexs(d)}\n" for a, d in cases) + "L -\n").decode().splitlines()
    assert len(text) == len(cases) + 1
    parts, nparts = [], []
    for ln in text[:-1]:
        c = ln.split(" ")
        assert c[0] == "P" and len(c) == int(c[1]) + 2
        nparts.append(int(c[1]))
        parts += [b"" if h == "-" else bytes.fromhex(h) for h in c[2:]]
    lay = text[-1].split(" ")
    assert lay[0] == "L"
    st_flat, st_off = cat([a for a, _ in cases])
    de_flat, de_off = cat([d for _, d in cases])
    pa_flat, pa_off = cat(parts)
    np.savez_compressed(os.path.join(HERE, "ref_split.npz"), strs=st_flat, str_off=st_off, delims=de_flat,
                        delim_off=de_off, parts=pa_flat, part_off=pa_off, nparts=np.array(nparts, np.int32),
                        layout=np.array([int(x) for x in lay[1:]], np.int32))

    blobs = fasta_inputs(rng)
    outs = {}
    for op in ("F", "S"):
        text = run([(op, b) for b in blobs])
        per = text.split(b"END\n")
        assert len(per) == len(blobs) + 1 and per[-1] == b""
        outs[op] = per[:-1]
    b_flat, b_off = cat(blobs)
    f_flat, f_off = cat(outs["F"])
    g_flat, g_off = cat(outs["S"])
    np.savez_compressed(os.path.join(HERE, "ref_fasta.npz"), blobs=b_flat, blob_off=b_off, out=f_flat, out_off=f_off,
                        sout=g_flat, sout_off=g_off)
    print(f"ref_windows: {len(seqs)} sequences, {len(w_flat)} windows; ref_split: {len(cases)} cases; "
          f"ref_fasta: {len(blobs)} blobs")


if __name__ == "__main__":
    sys.exit(main())
