"""ctypes wrapper of oracle/liboracle_skm.so -- TEST INFRASTRUCTURE (the checker).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.
See oracle/skm_oracle.cpp for what it restates (parity unpinned: no reference fixtures exist).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_PATH = os.path.join(ROOT, "oracle", "liboracle_skm.so")
STORED_DTYPE = np.dtype([("avg_from_end", "<u2"), ("function_index", "<u2"), ("mean", "<u2"),
                         ("median", "<u2"), ("var", "<u2")])
CALL_DTYPE = np.dtype([("start", "<u4"), ("end", "<u4"), ("count", "<i4"), ("function_index", "<u2"),
                       ("pad", "<u2"), ("protein_length_median", "<u4"),
                       ("protein_length_med_avg_dev", "<f4")])


class AnnotOpts(C.Structure):
    _fields_ = [("min_hits", C.c_int32), ("max_gap", C.c_int32), ("ignore_hypo", C.c_int32),
                ("hypo_index", C.c_int32), ("mean_mode", C.c_int32), ("mad_mode", C.c_int32)]


_lib = None


def olib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_PATH):
            subprocess.check_call(["make", "-C", ROOT, "oracle/liboracle_skm.so"])
        _lib = C.CDLL(ORACLE_PATH)
        P = C.c_void_p
        _lib.oracle_build.restype = C.c_int
        _lib.oracle_build.argtypes = [P, P, P, P, P, C.c_uint64, C.c_uint32, P, P, C.c_uint64, P, P, P, P, P]
        _lib.oracle_build_mt.restype = C.c_int
        _lib.oracle_build_mt.argtypes = [P, P, P, P, P, C.c_uint64, C.c_uint32, C.c_int, P, P, P, P, P, P, P]
        _lib.oracle_build_sel_mt.restype = C.c_int
        _lib.oracle_build_sel_mt.argtypes = [P, P, P, P, P, C.c_uint64, C.c_uint32, C.c_int, C.c_int, C.c_uint64, P, P,
                                             C.c_uint64, P, P, P, P, P, P, P, P]
        _lib.oracle_count_windows.restype = C.c_uint64
        _lib.oracle_count_windows.argtypes = [P, P, C.c_uint64]
        _lib.oracle_bdz_load.restype = P
        _lib.oracle_bdz_load.argtypes = [P, C.c_uint64]
        _lib.oracle_bdz_free.argtypes = [P]
        _lib.oracle_bdz_size.restype = C.c_uint32
        _lib.oracle_bdz_size.argtypes = [P]
        _lib.oracle_bdz_search_keys.argtypes = [P, P, C.c_uint64, P]
        _lib.oracle_jenkins_hash_vector.argtypes = [C.c_uint32, P, C.c_uint32, P]
        _lib.oracle_annotate.restype = C.c_int64
        _lib.oracle_annotate.argtypes = [P, P, P, P, P, C.c_uint64, C.POINTER(AnnotOpts), P, P, C.c_uint64]
        _lib.oracle_annotate_exact.restype = C.c_int64
        _lib.oracle_annotate_exact.argtypes = [P, P, C.c_uint64, P, P, P, C.c_uint64, C.POINTER(AnnotOpts), P, P,
                                               C.c_uint64]
        _lib.oracle_annotate_mt.restype = C.c_int64
        _lib.oracle_annotate_mt.argtypes = [P, P, P, P, P, C.c_uint64, C.POINTER(AnnotOpts), C.c_int]
        _lib.oracle_matrix_distance.restype = C.c_int64
        _lib.oracle_matrix_distance.argtypes = [P, P, P, P, P, P, C.c_uint64, C.c_int32, P, C.c_uint64]
        _lib.oracle_matrix_distance_mt.restype = C.c_int64
        _lib.oracle_matrix_distance_mt.argtypes = [P, P, P, P, P, P, C.c_uint64, C.c_int32, P, C.c_uint64, C.c_int]
        _lib.oracle_kmer_windows.restype = C.c_uint32
        _lib.oracle_kmer_windows.argtypes = [C.c_char_p, C.c_uint32, P]
        _lib.oracle_split.restype = C.c_uint64
        _lib.oracle_split.argtypes = [C.c_char_p, C.c_uint64, C.c_char_p, C.c_uint64, P, C.c_uint64]
        _lib.oracle_find_best_call.argtypes = [P, C.c_uint64, C.POINTER(C.c_char_p), C.c_uint64, P, P, P,
                                               C.c_char_p, C.c_uint64]
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def kmer_windows(seq: bytes) -> np.ndarray:
    """The window offsets the oracle's for_each_kmer<8> restatement yields over one sequence."""
    out = np.zeros(max(len(seq), 1), np.uint32)
    n = olib().oracle_kmer_windows(seq, len(seq), _p(out))
    return out[:n]


def split(s: bytes, delim: bytes) -> list:
    """The oracle's restatement of split() (operators.h:80-91)."""
    cap = len(s) + 2
    se = np.zeros(2 * cap, np.uint64)
    n = olib().oracle_split(s, len(s), delim, len(delim), _p(se), cap)
    return [s[int(se[2 * k]):int(se[2 * k + 1])] for k in range(n)]


def build(residues, seq_off, seq_len, seq_func, seq_id, n_functions):
    """Returns dict(keys, data, distinct_functions, seqs_with_func, n_seqs_with_signature,
    distinct_signatures) with keys sorted ascending."""
    L = olib()
    residues = np.ascontiguousarray(residues, np.uint8)
    seq_off = np.ascontiguousarray(seq_off, np.uint64)
    seq_len = np.ascontiguousarray(seq_len, np.uint32)
    seq_func = np.ascontiguousarray(seq_func, np.uint16)
    seq_id = np.ascontiguousarray(seq_id, np.uint32)
    n = len(seq_len)
    cap = int(L.oracle_count_windows(_p(seq_len), _p(seq_func), n)) + 1
    keys = np.zeros(cap, np.uint64)
    data = np.zeros(cap, STORED_DTYPE)
    df = np.zeros(max(n_functions, 1), np.uint32)
    sw = np.zeros(max(n_functions, 1), np.uint32)
    out_n = np.zeros(1, np.uint64)
    nsig = np.zeros(1, np.uint64)
    dsig = np.zeros(1, np.uint64)
    rc = L.oracle_build(_p(residues), _p(seq_off), _p(seq_len), _p(seq_func), _p(seq_id), n, n_functions,
                        _p(keys), _p(data), cap, _p(out_n), _p(df), _p(sw), _p(nsig), _p(dsig))
    assert rc == 0
    k = int(out_n[0])
    return dict(keys=keys[:k].copy(), data=data[:k].copy(), distinct_functions=df[:n_functions].copy(),
                seqs_with_func=sw[:n_functions].copy(), n_seqs_with_signature=int(nsig[0]),
                distinct_signatures=int(dsig[0]))


def build_mt(residues, seq_off, seq_len, seq_func, seq_id, n_functions, n_threads, sort=True):
    """oracle_build on n_threads host threads (CPU baseline); same results, keys sorted if sort."""
    L = olib()
    residues = np.ascontiguousarray(residues, np.uint8)
    seq_off = np.ascontiguousarray(seq_off, np.uint64)
    seq_len = np.ascontiguousarray(seq_len, np.uint32)
    seq_func = np.ascontiguousarray(seq_func, np.uint16)
    seq_id = np.ascontiguousarray(seq_id, np.uint32)
    n = len(seq_len)
    cap = int(L.oracle_count_windows(_p(seq_len), _p(seq_func), n)) + 1
    keys = np.empty(cap, np.uint64)
    data = np.empty(cap, STORED_DTYPE)
    df = np.zeros(max(n_functions, 1), np.uint32)
    sw = np.zeros(max(n_functions, 1), np.uint32)
    out_n = np.zeros(1, np.uint64)
    nsig = np.zeros(1, np.uint64)
    dsig = np.zeros(1, np.uint64)
    rc = L.oracle_build_mt(_p(residues), _p(seq_off), _p(seq_len), _p(seq_func), _p(seq_id), n, n_functions,
                           int(n_threads), _p(keys), _p(data), _p(out_n), _p(df), _p(sw), _p(nsig), _p(dsig))
    assert rc == 0
    k = int(out_n[0])
    keys, data = keys[:k], data[:k]
    if sort:
        o = np.argsort(keys, kind="stable")
        keys, data = keys[o], data[o]
    return dict(keys=keys.copy(), data=data.copy(), distinct_functions=df[:n_functions].copy(),
                seqs_with_func=sw[:n_functions].copy(), n_seqs_with_signature=int(nsig[0]),
                distinct_signatures=int(dsig[0]))


def slice_hash(keys: np.ndarray) -> np.ndarray:
    """MurmurHash3 fmix64 of little-endian keys (the output-slice hash, numpy)."""
    k = np.ascontiguousarray(keys, np.uint64).copy()
    with np.errstate(over="ignore"):
        k ^= k >> np.uint64(33)
        k *= np.uint64(0xff51afd7ed558ccd)
        k ^= k >> np.uint64(33)
        k *= np.uint64(0xc4ceb9fe1a85ec53)
        k ^= k >> np.uint64(33)
    return k


def build_slice_mt(residues, seq_off, seq_len, seq_func, seq_id, n_functions, n_threads, sel_bits, sel,
                   want_flags=False):
    """oracle_build_sel_mt: the build restricted to the keys of one output slice (fmix64 top
    sel_bits == sel) on n_threads host threads.  Returns the slice's kept k-mers (sorted), its
    distinct_functions / distinct_signatures / n_seqs_with_signature, the input's valid windows
    (all keys), the largest selected group and optionally per-sequence flags of the slice."""
    L = olib()
    residues = np.ascontiguousarray(residues, np.uint8)
    seq_off = np.ascontiguousarray(seq_off, np.uint64)
    seq_len = np.ascontiguousarray(seq_len, np.uint32)
    seq_func = np.ascontiguousarray(seq_func, np.uint16)
    seq_id = np.ascontiguousarray(seq_id, np.uint32)
    n = len(seq_len)
    w = int(L.oracle_count_windows(_p(seq_len), _p(seq_func), n))
    cap = 2 * (w >> sel_bits) + (1 << 20)  # kept <= selected windows (~ w / 2^sel_bits); retried if short
    while True:
        keys = np.empty(cap, np.uint64)
        data = np.empty(cap, STORED_DTYPE)
        df = np.zeros(max(n_functions, 1), np.uint32)
        sw = np.zeros(max(n_functions, 1), np.uint32)
        out_n, nsig, dsig, valid, mg = (np.zeros(1, np.uint64) for _ in range(5))
        flags = np.zeros(max(n, 1), np.uint8) if want_flags else None
        rc = L.oracle_build_sel_mt(_p(residues), _p(seq_off), _p(seq_len), _p(seq_func), _p(seq_id), n, n_functions,
                                   int(n_threads), int(sel_bits), int(sel), _p(keys), _p(data), cap, _p(out_n),
                                   _p(df), _p(sw), _p(nsig), _p(dsig), _p(valid), _p(mg),
                                   _p(flags) if flags is not None else None)
        k = int(out_n[0])
        if rc == 0:
            break
        cap = k + 1
    o = np.argsort(keys[:k], kind="stable")
    return dict(keys=keys[:k][o].copy(), data=data[:k][o].copy(), distinct_functions=df[:n_functions].copy(),
                seqs_with_func=sw[:n_functions].copy(), n_seqs_with_signature=int(nsig[0]),
                distinct_signatures=int(dsig[0]), valid_windows=int(valid[0]), max_group=int(mg[0]),
                flags=None if flags is None else flags[:n])


def count_windows(seq_len, seq_func) -> int:
    seq_len = np.ascontiguousarray(seq_len, np.uint32)
    seq_func = np.ascontiguousarray(seq_func, np.uint16)
    return int(olib().oracle_count_windows(_p(seq_len), _p(seq_func), len(seq_len)))


class Bdz:
    def __init__(self, mph_bytes: bytes):
        self._buf = np.frombuffer(mph_bytes, np.uint8).copy()
        self.h = olib().oracle_bdz_load(_p(self._buf), len(self._buf))
        assert self.h, "oracle could not parse the BDZ image"

    def size(self) -> int:
        return int(olib().oracle_bdz_size(self.h))

    def search(self, keys: np.ndarray) -> np.ndarray:
        keys = np.ascontiguousarray(keys, np.uint64)
        out = np.zeros(len(keys), np.uint32)
        olib().oracle_bdz_search_keys(self.h, _p(keys), len(keys), _p(out))
        return out

    def __del__(self):
        try:
            olib().oracle_bdz_free(self.h)
        except Exception:
            pass


def jenkins(seed: int, key: bytes):
    k = np.frombuffer(key, np.uint8).copy()
    out = np.zeros(3, np.uint32)
    olib().oracle_jenkins_hash_vector(seed, _p(k), len(k), _p(out))
    return [int(x) for x in out]


def annotate(bdz: Bdz, dat: bytes, residues, seq_off, seq_len, min_hits=5, max_gap=200, ignore_hypo=0,
             hypo_index=-1, mean_mode=0, mad_mode=0):
    residues = np.ascontiguousarray(residues, np.uint8)
    seq_off = np.ascontiguousarray(seq_off, np.uint64)
    seq_len = np.ascontiguousarray(seq_len, np.uint32)
    datb = np.frombuffer(dat, np.uint8).copy() if dat else np.zeros(10, np.uint8)
    n = len(seq_len)
    off = np.zeros(n + 1, np.uint64)
    cap = int(seq_len.astype(np.int64).sum()) + 16
    calls = np.zeros(cap, CALL_DTYPE)
    opts = AnnotOpts(min_hits, max_gap, ignore_hypo, hypo_index, mean_mode, mad_mode)
    tot = olib().oracle_annotate(bdz.h, _p(datb), _p(residues), _p(seq_off), _p(seq_len), n, C.byref(opts), _p(off),
                                 _p(calls), cap)
    assert tot >= 0
    return off, calls[:tot].copy()


def annotate_par(bdz: Bdz, dat: bytes, residues, seq_off, seq_len, n_threads, min_hits=5, max_gap=200,
                 ignore_hypo=0, hypo_index=-1, mean_mode=0, mad_mode=0):
    """annotate() (calls in CSR form) over contiguous sequence ranges on n_threads host threads:
    oracle_annotate releases the GIL, every range is the single-thread restatement."""
    from concurrent.futures import ThreadPoolExecutor
    residues = np.ascontiguousarray(residues, np.uint8)
    seq_off = np.ascontiguousarray(seq_off, np.uint64)
    seq_len = np.ascontiguousarray(seq_len, np.uint32)
    datb = np.frombuffer(dat, np.uint8).copy() if dat else np.zeros(10, np.uint8)
    n = len(seq_len)
    opts = AnnotOpts(min_hits, max_gap, ignore_hypo, hypo_index, mean_mode, mad_mode)
    T = max(1, int(n_threads))
    bounds = [n * t // (T * 4) for t in range(T * 4 + 1)]

    def one(t):
        a, b = bounds[t], bounds[t + 1]
        cap = 8 * (b - a) + 1024
        while True:
            off = np.zeros(b - a + 1, np.uint64)
            calls = np.zeros(cap, CALL_DTYPE)
            tot = olib().oracle_annotate(bdz.h, _p(datb), _p(residues), _p(seq_off[a:b].copy()),
                                         _p(seq_len[a:b].copy()), b - a, C.byref(opts), _p(off), _p(calls), cap)
            if tot >= 0:
                return off, calls[:tot]
            cap *= 4

    with ThreadPoolExecutor(T) as ex:
        parts = list(ex.map(one, range(T * 4)))
    offs = [np.zeros(1, np.uint64)]
    base = 0
    for off, calls in parts:
        offs.append(off[1:] + np.uint64(base))
        base += len(calls)
    return np.concatenate(offs), (np.concatenate([c for _, c in parts]) if parts else np.zeros(0, CALL_DTYPE))


def annotate_mt(bdz: Bdz, dat: bytes, residues, seq_off, seq_len, n_threads, min_hits=5, max_gap=200,
                ignore_hypo=0, hypo_index=-1, mean_mode=0, mad_mode=0) -> int:
    """process_aa_seq over every sequence on n_threads host threads; returns the number of calls."""
    residues = np.ascontiguousarray(residues, np.uint8)
    seq_off = np.ascontiguousarray(seq_off, np.uint64)
    seq_len = np.ascontiguousarray(seq_len, np.uint32)
    datb = np.frombuffer(dat, np.uint8).copy() if dat else np.zeros(10, np.uint8)
    opts = AnnotOpts(min_hits, max_gap, ignore_hypo, hypo_index, mean_mode, mad_mode)
    return int(olib().oracle_annotate_mt(bdz.h, _p(datb), _p(residues), _p(seq_off), _p(seq_len), len(seq_len),
                                         C.byref(opts), int(n_threads)))


def annotate_exact(keys, data, residues, seq_off, seq_len, min_hits=5, max_gap=200, ignore_hypo=0,
                   hypo_index=-1, mean_mode=0, mad_mode=0):
    """process_aa_seq against KeptKmerDB (exact keys; keys sorted ascending, data[i] for keys[i])."""
    keys = np.ascontiguousarray(keys, np.uint64)
    data = np.ascontiguousarray(data, STORED_DTYPE)
    residues = np.ascontiguousarray(residues, np.uint8)
    seq_off = np.ascontiguousarray(seq_off, np.uint64)
    seq_len = np.ascontiguousarray(seq_len, np.uint32)
    n = len(seq_len)
    off = np.zeros(n + 1, np.uint64)
    cap = int(seq_len.astype(np.int64).sum()) + 16
    calls = np.zeros(cap, CALL_DTYPE)
    opts = AnnotOpts(min_hits, max_gap, ignore_hypo, hypo_index, mean_mode, mad_mode)
    tot = olib().oracle_annotate_exact(_p(keys), _p(data), len(keys), _p(residues), _p(seq_off), _p(seq_len), n,
                                       C.byref(opts), _p(off), _p(calls), cap)
    assert tot >= 0
    return off, calls[:tot].copy()


def annotate_exact_par(keys, data, residues, seq_off, seq_len, n_threads, min_hits=5, max_gap=200, ignore_hypo=0,
                       hypo_index=-1, mean_mode=0, mad_mode=0):
    """annotate_exact() (the recall pass against KeptKmerDB, calls in CSR form) over contiguous
    sequence ranges on n_threads host threads: oracle_annotate_exact releases the GIL, every range
    is the single-thread restatement."""
    from concurrent.futures import ThreadPoolExecutor
    keys = np.ascontiguousarray(keys, np.uint64)
    data = np.ascontiguousarray(data, STORED_DTYPE)
    residues = np.ascontiguousarray(residues, np.uint8)
    seq_off = np.ascontiguousarray(seq_off, np.uint64)
    seq_len = np.ascontiguousarray(seq_len, np.uint32)
    n = len(seq_len)
    opts = AnnotOpts(min_hits, max_gap, ignore_hypo, hypo_index, mean_mode, mad_mode)
    T = max(1, int(n_threads))
    bounds = [n * t // (T * 4) for t in range(T * 4 + 1)]

    def one(t):
        a, b = bounds[t], bounds[t + 1]
        cap = 8 * (b - a) + 1024
        while True:
            off = np.zeros(b - a + 1, np.uint64)
            calls = np.zeros(cap, CALL_DTYPE)
            tot = olib().oracle_annotate_exact(_p(keys), _p(data), len(keys), _p(residues), _p(seq_off[a:b].copy()),
                                               _p(seq_len[a:b].copy()), b - a, C.byref(opts), _p(off), _p(calls), cap)
            if tot >= 0:
                return off, calls[:tot]
            cap *= 4

    with ThreadPoolExecutor(T) as ex:
        parts = list(ex.map(one, range(T * 4)))
    offs = [np.zeros(1, np.uint64)]
    base = 0
    for off, calls in parts:
        offs.append(off[1:] + np.uint64(base))
        base += len(calls)
    return np.concatenate(offs), (np.concatenate([c for _, c in parts]) if parts else np.zeros(0, CALL_DTYPE))


def matrix_distance_mt(bdz: Bdz, dat: bytes, residues, seq_off, seq_len, seq_idx, hypo_index=-1, n_threads=1,
                       want_pairs=True):
    """oracle_matrix_distance_mt: the pair counts on n_threads host threads; (n, 3) sorted pairs,
    or (want_pairs=False, the CPU baseline) only their number."""
    residues = np.ascontiguousarray(residues, np.uint8)
    seq_off = np.ascontiguousarray(seq_off, np.uint64)
    seq_len = np.ascontiguousarray(seq_len, np.uint32)
    seq_idx = np.ascontiguousarray(seq_idx, np.uint32)
    datb = np.frombuffer(dat, np.uint8).copy() if dat else np.zeros(10, np.uint8)
    L = olib()
    if not want_pairs:
        return int(L.oracle_matrix_distance_mt(bdz.h, _p(datb), _p(residues), _p(seq_off), _p(seq_len), _p(seq_idx),
                                               len(seq_len), hypo_index, None, 0, int(n_threads)))
    n = int(L.oracle_matrix_distance_mt(bdz.h, _p(datb), _p(residues), _p(seq_off), _p(seq_len), _p(seq_idx),
                                        len(seq_len), hypo_index, None, 0, int(n_threads)))
    out = np.zeros((max(n, 1), 3), np.uint32)
    L.oracle_matrix_distance_mt(bdz.h, _p(datb), _p(residues), _p(seq_off), _p(seq_len), _p(seq_idx), len(seq_len),
                                hypo_index, _p(out), n, int(n_threads))
    return out[:n].copy()


def matrix_distance(bdz: Bdz, dat: bytes, residues, seq_off, seq_len, seq_idx, hypo_index=-1):
    """kmers-matrix-distance pair counts: (n, 3) u32 array of (id1, id2, count), sorted."""
    residues = np.ascontiguousarray(residues, np.uint8)
    seq_off = np.ascontiguousarray(seq_off, np.uint64)
    seq_len = np.ascontiguousarray(seq_len, np.uint32)
    seq_idx = np.ascontiguousarray(seq_idx, np.uint32)
    datb = np.frombuffer(dat, np.uint8).copy() if dat else np.zeros(10, np.uint8)
    L = olib()
    n = int(L.oracle_matrix_distance(bdz.h, _p(datb), _p(residues), _p(seq_off), _p(seq_len), _p(seq_idx),
                                     len(seq_len), hypo_index, None, 0))
    out = np.zeros((max(n, 1), 3), np.uint32)
    L.oracle_matrix_distance(bdz.h, _p(datb), _p(residues), _p(seq_off), _p(seq_len), _p(seq_idx), len(seq_len),
                             hypo_index, _p(out), n)
    return out[:n].copy()


def find_best_call(calls: np.ndarray, function_index: list):
    calls = np.ascontiguousarray(calls, CALL_DTYPE)
    arr = (C.c_char_p * max(1, len(function_index)))(*[s.encode("latin-1") for s in function_index])
    fi = np.zeros(1, np.uint16)
    score = np.zeros(1, np.float32)
    off = np.zeros(1, np.float32)
    buf = C.create_string_buffer(4096)
    olib().oracle_find_best_call(_p(calls) if len(calls) else None, len(calls), arr, len(function_index), _p(fi),
                                 _p(score), _p(off), buf, 4096)
    return int(fi[0]), buf.value.decode("latin-1"), float(score[0]), float(off[0])
