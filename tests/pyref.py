"""Pure-Python restatement of the build and call-side window rules -- TEST INFRASTRUCTURE.

A second, independently written checker for SMALL inputs (dict grouping + Python loops), used to
cross-check the C++ oracle (oracle/skm_oracle.cpp) on randomized tiny cases.  It follows the same
reference lines:
  build_py        signature_build.tcc:121-181 (windows), :184-213 (group visit), :219-293 (cut/stats)
  P2              Boost.Accumulators p_square_quantile, p = 0.5
  call_windows    for_each_kmer, kmer_data.h:76-102
Parity with the reference itself is unpinned: the reference ships no fixtures.
"""
from __future__ import annotations

import struct

OK_PROT = set(b"ACDEFGHIKLMNPQRSTVWYacdefghiklmnpqrstvwy")  # signature_build.h:102-103


def d2u16(d: float) -> int:
    """(unsigned short) of a double as gcc/x86-64 emits it: cvttsd2si to int32, keep 16 bits."""
    if not (-2147483649.0 < d < 2147483648.0):
        return 0
    return int(d) & 0xFFFF  # int() truncates toward zero like cvttsd2si


class P2:
    """p_square_quantile with p = 0.5: heights, actual and desired marker positions."""

    def __init__(self):
        self.h = [0.0] * 5
        self.n = [1.0, 2.0, 3.0, 4.0, 5.0]
        self.d = [1.0, 2.0, 3.0, 4.0, 5.0]
        self.cnt = 0

    def add(self, x: int):
        self.cnt += 1
        x = float(x)
        if self.cnt <= 5:
            self.h[self.cnt - 1] = x
            if self.cnt == 5:
                self.h.sort()
            return
        h, n, d = self.h, self.n, self.d
        if x < h[0]:
            h[0] = x
            cell = 1
        elif x >= h[4]:
            h[4] = x
            cell = 4
        else:
            cell = next(k for k in range(5) if h[k] > x)  # upper_bound
        for k in range(cell, 5):
            n[k] += 1.0
        for k, inc in enumerate((0.0, 0.25, 0.5, 0.75, 1.0)):
            d[k] += inc
        for i in (1, 2, 3):
            di = d[i] - n[i]
            dp = n[i + 1] - n[i]
            dm = n[i - 1] - n[i]
            hp = (h[i + 1] - h[i]) / dp
            hm = (h[i - 1] - h[i]) / dm
            if (di >= 1.0 and dp > 1.0) or (di <= -1.0 and dm < -1.0):
                s = 1 if di > 0 else -1
                hh = h[i] + s / (dp - dm) * ((s - dm) * hp + (dp - s) * hm)
                if h[i - 1] < hh < h[i + 1]:
                    h[i] = hh
                elif di > 0:
                    h[i] = h[i] + hp
                else:
                    h[i] = h[i] - hm
                n[i] += s

    def result(self) -> float:
        return self.h[2]


def group_stats(lengths_in_visit_order):
    """accumulator_set<unsigned short, stats<mean, median, variance>> over the visit sequence."""
    cnt, s, var = 0, 0, 0.0
    p2 = P2()
    for x in lengths_in_visit_order:
        cnt += 1
        s = (s + x) & 0xFFFF
        p2.add(x)
        if cnt > 1:
            m = s / cnt
            t = x - m
            var = var * (cnt - 1) / cnt + t * t / (cnt - 1)
    mean = s / cnt
    return d2u16(mean), d2u16(p2.result()), d2u16(var)


def f32(x: float) -> float:
    return struct.unpack("<f", struct.pack("<f", x))[0]


def build_py(seqs, funcs, seq_ids, n_functions):
    """seqs: list of bytes; funcs: FunctionIndex per sequence (0xFFFF = skipped).
    Returns (dict key->(avg_from_end, func, mean, median, var), distinct_functions,
    seqs_with_func, n_seqs_with_signature)."""
    groups = {}
    seqs_with_func = [0] * n_functions
    for s, (seq, fn) in enumerate(zip(seqs, funcs)):
        if fn == 0xFFFF:
            continue
        seqs_with_func[fn] += 1
        for i in range(len(seq) - 7):
            w = seq[i:i + 8]
            if all(c in OK_PROT for c in w):
                key = int.from_bytes(w, "little")
                groups.setdefault(key, []).append((s, i))
    out = {}
    distinct = [0] * n_functions
    sig_seqs = set()
    for key, occ in groups.items():
        visit = occ[::-1]  # TBB 2020 multimap: reverse insertion order
        fc = {}
        for s, _ in visit:
            fc[funcs[s]] = fc.get(funcs[s], 0) + 1
        best_f, best_c = None, -1
        for fn in sorted(fc):
            if fc[fn] > best_c:
                best_f, best_c = fn, fc[fn]
        count = len(visit)
        if f32(float(best_c)) < f32(f32(float(count)) * f32(0.8)):
            continue
        lens = [len(seqs[s]) for s, _ in visit if funcs[s] == best_f]
        mean, med, var = group_stats(lens)
        offs = sorted((len(seqs[s]) - i) & 0xFFFF for s, i in visit)
        for s, _ in visit:
            sig_seqs.add(seq_ids[s])
        distinct[best_f] += 1
        out[key] = (offs[len(offs) // 2], best_f, mean, med, var)
    return out, distinct, seqs_with_func, len(sig_seqs)


def call_windows(seq: bytes):
    """for_each_kmer<8> (kmer_data.h:76-102): yields (offset, key) of the windows the call path
    looks up.  Only 'X' and '*' are ambiguous, and a window is also skipped when the ambiguous
    character sits immediately after it (next_ambig <= ptr + 8)."""
    n = len(seq)
    out = []
    p = 0
    while p + 8 <= n:
        nxt = next((q for q in range(p, n) if seq[q] in b"X*"), n)
        if nxt <= p + 8 and nxt < n:
            p = nxt + 1
            continue
        out.append((p, int.from_bytes(seq[p:p + 8], "little")))
        p += 1
    return out


def matrix_distance(seqs, seq_idx, fetch, hypo_index):
    """kmers-matrix-distance (kmers-matrix-distance.cc:123-196): every window of for_each_kmer whose
    record (fetch(key) -> (avg, func, mean, median, var) or None) is not hypothetical and whose
    sequence length lies within mean -/+ 2 sd (sd = sqrt(var), or 0.1 * seqlen when var == 0) adds
    the sequence's index to the k-mer's set; every pair id1 < id2 of a set counts once.
    Returns {(id1, id2): count}."""
    import math
    sets = {}
    for s, seq in enumerate(seqs):
        seqlen = float(len(seq))
        for _, key in call_windows(seq):
            kd = fetch(key)
            if kd is None or kd[1] == hypo_index:
                continue
            mean = float(kd[2])
            sd = seqlen * 0.1 if kd[4] == 0 else math.sqrt(float(kd[4]))
            if seqlen < mean - sd * 2.0 or seqlen > mean + sd * 2.0:
                continue
            sets.setdefault(key, set()).add(int(seq_idx[s]))
    dist = {}
    for ids in sets.values():
        v = sorted(ids)
        for a in range(len(v)):
            for b in range(a + 1, len(v)):
                dist[(v[a], v[b])] = dist.get((v[a], v[b]), 0) + 1
    return dist
