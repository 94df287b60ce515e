"""CPU restatement of the CLI front end -- TEST INFRASTRUCTURE (the checker).

Only tests/ import this module; the product CLIs (signature_kmers_amd/csrc/tools, front/) never
do.  It restates, with Python's `re` (Perl-style backtracking, the same leftmost-first semantics
as Boost.Regex's Perl mode) instead of the hand-coded matchers the C++ front end uses:

  FastaParser                       fasta_parser.h:38-144, fasta_parser.cc:17-36
  seed_utils regexes                seed_utils.h:10-62
  FunctionMap                       function_map.h:62-411 (load_id_assignments, load_fasta_file,
                                    process_kept_functions, write_function_index)
  SignatureBuilder::load_kmers_from_fasta / _sequence   signature_build.tcc:84-181
  accumulator_set<float, mean, median(P^2), variance, count>   (function.index columns 2-6)
  the recall report                 kmers-build-signatures.cc:238-349
  kmers-call-functions / kmers-annotate-seqs output     kmers-call-functions.cc:167-181,
                                    kmers-annotate-seqs.cc:136-167

Parity: unpinned by the reference (it ships no tests or fixtures).  Boost.Regex,
Boost.Accumulators and the x86 "-nan" printing of an empty accumulator's mean are restated from
their documented semantics.
"""
from __future__ import annotations

import math
import os
import re

import numpy as np

MAX_SEQS_PER_FILE = 100000
UNDEF = 0xFFFF

_WS = rb"[ \t\n\v\f\r]"
RE_SPLIT_FUNC_COMMENT = re.compile(rb"(.*?)(?:" + _WS + rb"+(#+)" + _WS + rb"+(.*))?", re.S)
RE_TRUNC = re.compile(rb"^(?:frag|missing|trunc)", re.M)
RE_STRIP_COMMENT = re.compile(_WS + rb"*#.*$", re.S)
RE_SPLIT_FUNCTION = re.compile(_WS + rb"+[/@]" + _WS + rb"+|" + _WS + rb"*;" + _WS + rb"+")
RE_GENOME = re.compile(_WS + rb"+(.*)" + _WS + rb"+\[([^]]+)\]$", re.S)
RE_FIGID = re.compile(rb"fig\|([0-9]+\.[0-9]+)")
RE_GENOME_ID = re.compile(rb"[0-9]+\.[0-9]+")


# ------------------------------------------------------------------------------------------
# FASTA
# ------------------------------------------------------------------------------------------
def parse_fasta(data: bytes):
    """[(id, def, seq)] for records with a non-empty id (callers skip empty ids)."""
    out = []
    st = 0  # 0 start, 1 id, 2 defline, 3 data, 4 id_or_data
    cid, cdef, cseq = bytearray(), bytearray(), bytearray()

    def emit():
        if cid:
            out.append((bytes(cid), bytes(cdef), bytes(cseq)))

    for c in data:
        if c == 13:
            continue
        if st == 0:
            if c == 62:
                st = 1
        elif st == 1:
            if c in (32, 9):
                cdef.append(c)
                st = 2
            elif c == 10:
                st = 3
            else:
                cid.append(c)
        elif st == 2:
            if c == 10:
                st = 3
            else:
                cdef.append(c)
        elif st == 3:
            if c == 10:
                st = 4
            elif (65 <= c <= 90) or (97 <= c <= 122) or c == 42:
                cseq.append(c)
        else:
            if c == 62:
                emit()
                cid, cdef, cseq = bytearray(), bytearray(), bytearray()
                st = 1
            elif c == 10:
                pass
            elif (65 <= c <= 90) or (97 <= c <= 122):
                cseq.append(c)
                st = 3
    emit()
    return out


# ------------------------------------------------------------------------------------------
# seed_utils
# ------------------------------------------------------------------------------------------
def split_func_comment(s: bytes):
    m = RE_SPLIT_FUNC_COMMENT.fullmatch(s)
    return m.group(1), m.group(2) or b"", m.group(3) or b""


def is_truncated_comment(s: bytes) -> bool:
    return RE_TRUNC.search(s) is not None


def strip_func_comment(s: bytes) -> bytes:
    return RE_STRIP_COMMENT.sub(b"", s)


def roles_of_function(f: bytes):
    s = strip_func_comment(f)
    toks, last, any_m = [], 0, False
    for m in RE_SPLIT_FUNCTION.finditer(s):
        toks.append(s[last:m.start()])
        last = m.end()
        any_m = True
    if not any_m:
        return [s] if s else []
    if last != len(s):
        toks.append(s[last:])
    return toks


def match_genome(defl: bytes):
    m = RE_GENOME.fullmatch(defl)
    return (m.group(1), m.group(2)) if m else None


# ------------------------------------------------------------------------------------------
# accumulator_set<float, stats<mean, median, variance, count>>
# ------------------------------------------------------------------------------------------
F = np.float32


class FloatStats:
    INCR = [F(0.0), F(0.25), F(0.5), F(0.75), F(1.0)]

    def __init__(self):
        self.count = 0
        self.sum = F(0)
        self.var = F(0)
        self.h = [F(0)] * 5
        self.act = [F(1), F(2), F(3), F(4), F(5)]
        self.des = [F(1), F(2), F(3), F(4), F(5)]

    def add(self, x):
        x = F(x)
        self.count += 1
        n = self.count
        self.sum = F(self.sum + x)
        h, act, des = self.h, self.act, self.des
        if n <= 5:
            h[n - 1] = x
            if n == 5:
                h.sort()
        else:
            if x < h[0]:
                h[0] = x
                cell = 1
            elif h[4] <= x:
                h[4] = x
                cell = 4
            else:
                cell = next(i for i in range(5) if h[i] > x)
            for i in range(cell, 5):
                act[i] = F(act[i] + F(1))
            for i in range(5):
                des[i] = F(des[i] + self.INCR[i])
            for i in (1, 2, 3):
                d = F(des[i] - act[i])
                dp = F(act[i + 1] - act[i])
                dm = F(act[i - 1] - act[i])
                hp = F(F(h[i + 1] - h[i]) / dp)
                hm = F(F(h[i - 1] - h[i]) / dm)
                if (d >= 1.0 and dp > 1) or (d <= -1.0 and dm < -1):
                    sd = 1 if d > 0 else -1
                    sdf = F(sd)
                    hh = F(h[i] + F(F(sdf / F(dp - dm)) * F(F(F(sdf - dm) * hp) + F(F(dp - sdf) * hm))))
                    if h[i - 1] < hh < h[i + 1]:
                        h[i] = hh
                    else:
                        if d > 0:
                            h[i] = F(h[i] + hp)
                        if d < 0:
                            h[i] = F(h[i] - hm)
                    act[i] = F(act[i] + sdf)
        if n > 1:
            mean = F(self.sum / F(n))
            tmp = F(x - mean)
            self.var = F(F(F(self.var * F(n - 1)) / F(n)) + F(F(tmp * tmp) / F(n - 1)))


def fmt_g(v) -> str:
    v = float(v)
    if math.isnan(v):
        return "-nan" if math.copysign(1.0, v) < 0 else "nan"
    if math.isinf(v):
        return "-inf" if v < 0 else "inf"
    return "%g" % v


# ------------------------------------------------------------------------------------------
# FunctionMap + sequence selection
# ------------------------------------------------------------------------------------------
class FunctionMapRef:
    def __init__(self, good_functions=(), good_roles=()):
        self.fgm = {}           # function -> set(genome)
        self.idf = {}           # id -> function
        self.orig = {}
        self.orig_stripped = {}
        self.acc = {}
        self.good_functions = set(good_functions)
        self.good_roles = set(good_roles)
        self.fidx = {}
        self.idxf = {}

    def load_id_assignments(self, path):
        with open(path, "rb") as fh:
            data = fh.read()
        lines = data.split(b"\n")
        if lines and lines[-1] == b"":
            lines.pop()
        for line in lines:
            s = line.find(b"\t")
            if s < 0:
                continue
            s2 = line.find(b"\t", s + 1)
            pid = line[:s]
            func = line[s + 1:] if s2 < 0 else line[s + 1:s2]
            stripped, delim, comment = split_func_comment(func)
            self.orig_stripped[pid] = stripped
            self.orig[pid] = func
            if delim == b"#" and is_truncated_comment(comment):
                continue
            self.idf[pid] = stripped

    def load_fasta_records(self, filename: bytes, records, deleted):
        genome = b""
        for pid, defl, seq in records:
            if pid in deleted:
                continue
            func = b""
            if defl:
                stripped = defl.lstrip(b" \t")
                if not stripped:
                    raise ValueError("blank definition line")
                func = stripped
            gl = b""
            m = match_genome(defl)
            if m:
                func, delim, comment = split_func_comment(m[0])
                if delim == b"#" and is_truncated_comment(comment):
                    continue
                gl = m[1]
            if not genome:
                if not defl:
                    mm = RE_FIGID.search(pid)
                    if mm:
                        genome = mm.group(1)
                elif gl:
                    genome = gl
            if not genome:
                genome = filename
            cur = self.idf.get(pid, b"")
            if not cur:
                self.idf[pid] = func
            else:
                func = cur
            if func:
                self.fgm.setdefault(func, set()).add(genome)
                self.acc.setdefault(func, FloatStats()).add(len(seq))

    def process_kept_functions(self, min_reps, ignored):
        kept = set()
        for f in sorted(self.fgm):
            ok = len(self.fgm[f]) >= min_reps or f in self.good_functions
            if not ok:
                ok = any(r in self.good_roles for r in roles_of_function(f))
            if ok:
                kept.add(f)
        kept.add(b"hypothetical protein")
        for f in ignored:
            kept.discard(f)
        self.fidx = {f: i for i, f in enumerate(sorted(kept))}
        self.idxf = {i: f for f, i in self.fidx.items()}
        return len(kept)

    def function_index_text(self) -> bytes:
        out = []
        for i in sorted(self.idxf):
            f = self.idxf[i]
            a = self.acc.setdefault(f, FloatStats())
            if a.count == 0:
                mean = "-nan"  # 0.0f / 0 on x86 = the default NaN (sign bit set)
            else:
                mean = fmt_g(F(a.sum / F(a.count)))
            var = float(a.var)
            out.append(b"%d\t%s\t%d\t%s\t%s\t%s\t%s\n" % (i, f, a.count, mean.encode(), fmt_g(a.h[2]).encode(),
                                                          fmt_g(var).encode(), fmt_g(math.sqrt(var)).encode()))
        return b"".join(out)


def list_files(d):
    """directory_iterator order (readdir), regular files only."""
    out = []
    with os.scandir(d) as it:
        for e in it:
            if e.is_file():
                out.append(os.path.join(d, e.name))
    return out


def read_lines(path):
    with open(path, "rb") as fh:
        lines = fh.read().split(b"\n")
    if lines and lines[-1] == b"":
        lines.pop()
    return lines


def front(definition_dirs, fasta_dirs, keep_dirs=(), good_functions=(), good_roles=(), deleted=(), ignored=(),
          min_reps=3, records=None):
    """Run the reference front end.  Returns dict(fm, files=[(path, records)], build=(residues, off, len,
    func, seq_id), n_kept_functions).  records: {path: [(id, def, seq)]} to use instead of parsing
    those files (callers that know what FastaParser yields for them, e.g. generated files)."""
    fm = FunctionMapRef(good_functions, good_roles)
    for d in definition_dirs:
        for p in list_files(d):
            fm.load_id_assignments(p)
    deleted = set(deleted)
    paths = [p for d in fasta_dirs for p in list_files(d)] + [p for d in keep_dirs for p in list_files(d)]
    files = []
    for p in paths:
        if records is not None and p in records:
            recs = records[p]
        else:
            with open(p, "rb") as fh:
                recs = parse_fasta(fh.read())
        files.append((p, recs))
        fm.load_fasta_records(os.path.basename(p).encode(), recs, deleted)
    nk = fm.process_kept_functions(min_reps, set(ignored))
    res, off, ln, fn, sid = bytearray(), [], [], [], []
    for fnum, (p, recs) in enumerate(files):
        nxt = (fnum * MAX_SEQS_PER_FILE) & 0xFFFFFFFF
        for pid, defl, seq in recs:
            if pid in deleted:
                continue
            func = fm.idf.get(pid, b"")
            if not func:
                continue
            seq_id = nxt
            nxt = (nxt + 1) & 0xFFFFFFFF
            fi = fm.fidx.get(func, UNDEF)
            if fi == UNDEF:
                continue
            off.append(len(res))
            res += seq
            ln.append(len(seq))
            fn.append(fi)
            sid.append(seq_id)
    build = (np.frombuffer(bytes(res), np.uint8).copy(), np.array(off, np.uint64), np.array(ln, np.uint32),
             np.array(fn, np.uint16), np.array(sid, np.uint32))
    return dict(fm=fm, files=files, build=build, n_kept_functions=nk)


def read_dump(path):
    """--dump-extract file of bin/kmers-build-signatures."""
    with open(path, "rb") as fh:
        b = fh.read()
    n, nr = np.frombuffer(b[:16], np.uint64)
    n, nr = int(n), int(nr)
    p = 16
    res = np.frombuffer(b[p:p + nr], np.uint8)
    p += nr
    off = np.frombuffer(b[p:p + 8 * n], np.uint64)
    p += 8 * n
    ln = np.frombuffer(b[p:p + 4 * n], np.uint32)
    p += 4 * n
    fn = np.frombuffer(b[p:p + 2 * n], np.uint16)
    p += 2 * n
    sid = np.frombuffer(b[p:p + 4 * n], np.uint32)
    return res, off, ln, fn, sid


def records_arrays(recs):
    res = b"".join(r[2] for r in recs)
    ln = np.array([len(r[2]) for r in recs], np.uint32)
    off = np.zeros(len(recs), np.uint64)
    if len(recs):
        off[1:] = np.cumsum(ln[:-1].astype(np.uint64))
    return np.frombuffer(res, np.uint8).copy(), off, ln


def calls_per_record(oref, recs, function_index, exact=None, bdz=None, dat=None, ignore_hypo=False):
    """[(fi, func, score)] per record: process_aa_seq (exact kept-k-mer DB or BDZ) + find_best_call."""
    hypo = function_index.index("hypothetical protein")
    res, off, ln = records_arrays(recs)
    if exact is not None:
        coff, calls = oref.annotate_exact(exact[0], exact[1], res, off, ln, ignore_hypo=int(ignore_hypo),
                                          hypo_index=hypo)
    else:
        coff, calls = oref.annotate(bdz, dat, res, off, ln, ignore_hypo=int(ignore_hypo), hypo_index=hypo)
    out = []
    for s in range(len(recs)):
        fi, func, score, _ = oref.find_best_call(calls[int(coff[s]):int(coff[s + 1])], function_index)
        out.append((fi, func, score))
    return out


def recall_report(oref, fm: FunctionMapRef, recs, function_index, keys, data) -> bytes:
    """recall.report.d/<file> (kmers-build-signatures.cc:279-349)."""
    got = {}
    for (pid, _, _), (fi, func, score) in zip(recs, calls_per_record(oref, recs, function_index, exact=(keys, data))):
        o = fm.orig.get(pid, b"")
        os_ = fm.orig_stripped.get(pid, b"")
        if os_ != func.encode("latin-1") and pid not in got:
            got[pid] = b"%s\t%s\t%s\t%s\t%d\t%s\n" % (pid, o, os_, func.encode("latin-1"), fi, fmt_g(score).encode())
    return b"".join(got[k] for k in sorted(got))


def call_lines(oref, recs, function_index, bdz, dat, ignore_hypo=False, annotate_mode=False):
    out, uncalled = [], []
    for (pid, _, _), (fi, func, score) in zip(recs, calls_per_record(oref, recs, function_index, bdz=bdz, dat=dat,
                                                                    ignore_hypo=ignore_hypo)):
        if annotate_mode and fi == UNDEF:
            uncalled.append(pid + b"\n")
            continue
        out.append(b"%s\t%s\t%d\t%s\n" % (pid, func.encode("latin-1"), fi, fmt_g(score).encode()))
    return b"".join(out), b"".join(uncalled)
