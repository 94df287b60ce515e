"""signature_kmers_amd -- MI355X-native signature-k-mer engine (host mirror over libskm's C-ABI).

The reference (olsonanl/signature_kmers) exposes its hot path as C++ templates:
``SignatureBuilder<8>`` (signature_build.h:55-147), the KmerDb concept ``CmphKmerDb``
(cmph_kmer.h:28-164) and ``FunctionCaller<KmerDb>`` (call_functions.h:60-136).  This module
mirrors those classes in Python on top of ``libskm.so`` (include/skm.h).  Every compute call goes
to the HIP library; there is no CPU fallback -- a missing library raises immediately.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

__all__ = [
    "SkmError", "lib", "K", "UNDEFINED_FUNCTION", "STORED_DTYPE", "CALL_DTYPE",
    "SignatureBuilder", "KeptKmers", "CmphKmerDb", "FunctionCaller", "mph_build",
    "kmer_to_str", "str_to_kmer", "keys_from_strings", "device_count", "MatrixDistance", "SeqIdMap",
    "matrix_tile_rows",
]

K = 8
UNDEFINED_FUNCTION = 0xFFFF
_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SKM_LIB_PATH") or os.path.join(_HERE, "libskm.so")  # override: A/B builds

STORED_DTYPE = np.dtype([("avg_from_end", "<u2"), ("function_index", "<u2"), ("mean", "<u2"),
                         ("median", "<u2"), ("var", "<u2")])  # StoredKmerData, kmer_data.h:114-128
CALL_DTYPE = np.dtype([("start", "<u4"), ("end", "<u4"), ("count", "<i4"), ("function_index", "<u2"),
                       ("pad", "<u2"), ("protein_length_median", "<u4"),
                       ("protein_length_med_avg_dev", "<f4")])  # KmerCall, call_functions.h:23-48


class SkmError(RuntimeError):
    pass


class _BuildOpts(C.Structure):
    _fields_ = [("k", C.c_int32), ("max_seqs_per_file", C.c_uint32), ("n_functions", C.c_uint32),
                ("canonical_order", C.c_int32), ("rank", C.c_int32), ("world_size", C.c_int32)]


_A2A_T = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.c_void_p,
                     C.POINTER(C.c_uint64), C.POINTER(C.c_uint64))
_RED_T = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_uint64, C.c_int)
_AGV_T = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64))


class _Transport(C.Structure):
    _fields_ = [("ctx", C.c_void_p), ("alltoallv", _A2A_T), ("allreduce", _RED_T), ("allgatherv", _AGV_T)]


class _Kept(C.Structure):
    _fields_ = [("keys", C.POINTER(C.c_uint64)), ("data", C.c_void_p), ("n", C.c_uint64),
                ("distinct_functions", C.POINTER(C.c_uint32)), ("seqs_with_func", C.POINTER(C.c_uint32)),
                ("n_functions", C.c_uint32), ("n_seqs_with_signature", C.c_uint64),
                ("distinct_signatures", C.c_uint64), ("n_windows", C.c_uint64), ("n_records", C.c_uint64)]


class _AnnotOpts(C.Structure):
    _fields_ = [("min_hits", C.c_int32), ("max_gap", C.c_int32), ("ignore_hypo", C.c_int32),
                ("hypo_index", C.c_int32), ("mean_mode", C.c_int32), ("mad_mode", C.c_int32)]


class _Calls(C.Structure):
    _fields_ = [("call_off", C.POINTER(C.c_uint64)), ("calls", C.c_void_p), ("n_seqs", C.c_uint64),
                ("n_calls", C.c_uint64), ("n_windows", C.c_uint64)]


class _MatrixOpts(C.Structure):
    _fields_ = [("hypo_index", C.c_int32), ("row_begin", C.c_uint32), ("row_end", C.c_uint32), ("pad", C.c_uint32),
                ("max_tile_bytes", C.c_uint64)]


class _Pairs(C.Structure):
    _fields_ = [("pairs", C.POINTER(C.c_uint32)), ("n", C.c_uint64), ("n_hits", C.c_uint64)]


_P = C.c_void_p
_SIGS = {
    "skm_last_error": (C.c_char_p, []),
    "skm_version": (C.c_char_p, []),
    "skm_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "skm_build_create": (C.c_int, [C.POINTER(_P), C.POINTER(C.c_int), C.c_int, C.POINTER(_BuildOpts)]),
    "skm_build_add_batch": (C.c_int, [_P, _P, _P, _P, _P, _P, C.c_size_t]),
    "skm_build_prepare": (C.c_int, [_P]),
    "skm_build_run": (C.c_int, [_P]),
    "skm_build_last_timings": (C.c_int, [_P, C.POINTER(C.c_float), C.c_int]),
    "skm_build_set_kernel_timing": (C.c_int, [_P, C.c_int, C.c_char_p]),
    "skm_build_kernel_timings": (C.c_int, [_P, C.c_char_p, C.c_size_t, C.POINTER(C.c_float), C.POINTER(C.c_uint64),
                                           C.c_int]),
    "skm_build_finish": (C.c_int, [_P, C.POINTER(_Kept)]),
    "skm_build_finish_slice": (C.c_int, [_P, C.c_int, C.c_uint32, C.POINTER(_Kept)]),
    "skm_build_signature_flags": (C.c_int, [_P, _P, C.c_uint64]),
    "skm_build_set_option": (C.c_int, [_P, C.c_char_p, C.c_int64]),
    "skm_build_set_transport": (C.c_int, [_P, C.POINTER(_Transport)]),
    "skm_debug_exchange_plan": (C.c_int, [C.POINTER(_Transport), C.c_int, C.c_int, C.c_uint32, _P, _P, _P, _P]),
    "skm_debug_transport_check": (C.c_int, [C.POINTER(_Transport), C.c_int, C.c_int]),
    "skm_build_counters": (C.c_int, [_P, C.POINTER(C.c_uint64), C.c_int]),
    "skm_build_reserve": (C.c_int, [_P, C.c_uint64, C.c_uint64]),
    "skm_build_debug_jobs": (C.c_int, [_P, C.POINTER(C.c_uint32), C.c_int]),
    "skm_build_debug_overflow": (C.c_int, [_P, C.POINTER(C.c_uint32), C.c_int]),
    "skm_debug_chain_bench": (C.c_int, [C.c_uint32, C.c_uint32, C.c_int, C.POINTER(C.c_float)]),
    "skm_debug_chain_eval": (C.c_int, [_P, C.c_uint32, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    "skm_build_debug_stamps": (C.c_int, [_P, C.c_int, C.POINTER(C.c_uint64), C.c_int]),
    "skm_kept_free": (None, [C.POINTER(_Kept)]),
    "skm_build_destroy": (None, [_P]),
    "skm_comm_unique_id": (C.c_int, [_P]),
    "skm_build_set_comm": (C.c_int, [_P, _P]),
    "skm_build_group_run": (C.c_int, [C.POINTER(_P), C.c_int]),
    "skm_debug_div_check": (C.c_int, [C.c_uint64, C.c_uint32, C.POINTER(C.c_uint64)]),
    "skm_db_open": (C.c_int, [C.POINTER(_P), C.c_char_p, C.c_char_p, C.c_int]),
    "skm_db_open_mem": (C.c_int, [C.POINTER(_P), _P, C.c_size_t, _P, C.c_size_t, C.c_int]),
    "skm_db_open_kept": (C.c_int, [C.POINTER(_P), _P, _P, C.c_size_t, C.c_int]),
    "skm_db_size": (C.c_int, [_P, C.POINTER(C.c_uint32)]),
    "skm_db_lookup": (C.c_int, [_P, _P, C.c_size_t, _P]),
    "skm_debug_db_lookup_generic": (C.c_int, [_P, _P, C.c_size_t, _P]),
    "skm_db_close": (None, [_P]),
    "skm_mph_build": (C.c_int, [_P, _P, C.c_size_t, C.c_uint32, C.c_char_p, C.c_char_p]),
    "skm_mph_build_device": (C.c_int, [_P, _P, C.c_size_t, C.c_uint32, C.c_char_p, C.c_char_p, C.c_int]),
    "skm_mph_build_device_ex": (C.c_int, [_P, _P, C.c_size_t, C.c_uint32, C.c_char_p, C.c_char_p, C.c_int, C.c_int,
                                          C.c_void_p]),
    "skm_query_create": (C.c_int, [C.POINTER(_P), _P, _P, _P, _P, C.c_size_t]),
    "skm_query_run": (C.c_int, [_P, C.POINTER(_AnnotOpts)]),
    "skm_query_last_timings": (C.c_int, [_P, C.POINTER(C.c_float), C.c_int]),
    "skm_query_calls": (C.c_int, [_P, C.POINTER(_Calls)]),
    "skm_query_window_hits": (C.c_int, [_P, _P, _P, _P, C.c_uint64, C.POINTER(C.c_uint64)]),
    "skm_query_destroy": (None, [_P]),
    "skm_annotate": (C.c_int, [_P, _P, _P, _P, C.c_size_t, C.POINTER(_AnnotOpts), C.POINTER(_Calls)]),
    "skm_calls_free": (None, [C.POINTER(_Calls)]),
    "skm_matrix_create": (C.c_int, [C.POINTER(_P), _P, _P, _P, _P, _P, C.c_size_t, C.c_uint32]),
    "skm_matrix_run": (C.c_int, [_P, C.POINTER(_MatrixOpts)]),
    "skm_matrix_set_transport": (C.c_int, [_P, C.c_int, C.c_int, C.POINTER(_Transport)]),
    "skm_matrix_set_comm": (C.c_int, [_P, C.c_int, C.c_int, _P]),
    "skm_matrix_last_timings": (C.c_int, [_P, C.POINTER(C.c_float), C.c_int]),
    "skm_matrix_counters": (C.c_int, [_P, C.POINTER(C.c_uint64), C.c_int]),
    "skm_matrix_pairs": (C.c_int, [_P, C.POINTER(_Pairs)]),
    "skm_pairs_free": (None, [C.POINTER(_Pairs)]),
    "skm_matrix_destroy": (None, [_P]),
    "skm_matrix_tile_rows": (C.c_int, [C.c_uint32, C.c_int, C.c_int, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
    "skm_find_best_call": (C.c_int, [_P, C.c_size_t, C.POINTER(C.c_char_p), C.c_size_t, C.POINTER(C.c_uint16),
                                     C.POINTER(C.c_float), C.POINTER(C.c_float), C.c_char_p, C.c_size_t]),
}

_lib = None


def lib():
    """Load libskm.so (built in-tree by __graft_entry__.build / `make`).  Fails loudly."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise SkmError(f"{LIB_PATH} is missing: run `make` (or __graft_entry__.build()) first")
        h = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(h, name)
            fn.restype = res
            fn.argtypes = args
        _lib = h
    return _lib


def _check(rc: int):
    if rc != 0:
        raise SkmError(f"libskm error {rc}: {lib().skm_last_error().decode(errors='replace')}")


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def debug_chain_bench(n: int, njobs: int, mode: int = 0) -> float:
    ms = C.c_float()
    _check(lib().skm_debug_chain_bench(n, njobs, mode, C.byref(ms)))
    return ms.value


def debug_chain_eval(samples, mode: int):
    """(P^2 median, variance) as raw doubles for one chain (samples in visit order)."""
    x = np.ascontiguousarray(samples, dtype=np.uint32)
    med, var = C.c_double(), C.c_double()
    _check(lib().skm_debug_chain_eval(_ptr(x), len(x), mode, C.byref(med), C.byref(var)))
    return med.value, var.value


def debug_div_check(nm: int, per: int) -> int:
    """Mismatches of the device exact-division helpers against IEEE division."""
    v = C.c_uint64(0)
    _check(lib().skm_debug_div_check(nm, per, C.byref(v)))
    return v.value


def device_count() -> int:
    n = C.c_int(0)
    _check(lib().skm_device_count(C.byref(n)))
    return n.value


def warm_device(device: int = 0) -> None:
    """Bring up the process's HIP runtime and the device context (one throwaway build handle), so
    that a timed one-shot build does not include the runtime's start-up."""
    SignatureBuilder(1, device=device).close()


def kmer_to_str(key: int) -> str:
    return int(key).to_bytes(8, "little").decode("latin-1")


def str_to_kmer(s: str) -> int:
    b = s.encode("latin-1")
    assert len(b) == K
    return int.from_bytes(b, "little")


def keys_from_strings(strs) -> np.ndarray:
    return np.array([str_to_kmer(s) for s in strs], dtype=np.uint64)


@dataclass
class KeptKmers:
    """KeptKmers<8> + KmerStatistics (signature_build.h:34-53), keys sorted ascending."""
    keys: np.ndarray                 # u64 little-endian k-mers
    data: np.ndarray                 # STORED_DTYPE
    distinct_functions: np.ndarray   # u32[n_functions]
    seqs_with_func: np.ndarray       # u32[n_functions]
    n_seqs_with_signature: int
    distinct_signatures: int
    n_windows: int

    def stats_lines(self) -> str:
        """stdout of process_kmers (signature_build.tcc:210-212)."""
        return (f"Kept {len(self.keys)} kmers\ndistinct_signatures={self.distinct_signatures}\n"
                f"num_seqs_with_a_signature={self.n_seqs_with_signature}\n")

    def final_kmers_lines(self):
        """final.kmers rows (kmers-build-signatures.cc:212-216): KMER \\t avg_from_end \\t fi \\t"""
        for k, d in zip(self.keys, self.data):
            yield f"{kmer_to_str(k)}\t{int(d['avg_from_end'])}\t{int(d['function_index'])}\t\n"


class _KeptOwner:
    """Owns one skm_kept's library arrays; frees them when the last numpy view is gone."""

    def __init__(self, k):
        self.k = k

    def __del__(self):
        try:
            lib().skm_kept_free(C.byref(self.k))
        except Exception:
            pass


class SignatureBuilder:
    """Device signature build (SignatureBuilder<8>::extract_kmers + process_kmers).

    Sequences are added in reference emission order with their FunctionIndex (0xFFFF = no kept
    function) and seq_id (file_number * max_seqs_per_file + k)."""

    def __init__(self, n_functions: int, max_seqs_per_file: int = 100000, device: int = 0, rank: int = 0,
                 world_size: int = 1):
        self._h = C.c_void_p()
        opts = _BuildOpts(8, max_seqs_per_file, n_functions, 1, rank, world_size)
        self.rank, self.world_size = rank, world_size
        dev = (C.c_int * 1)(device)
        _check(lib().skm_build_create(C.byref(self._h), dev, 1, C.byref(opts)))
        self.n_functions = n_functions

    def add_batch(self, residues, seq_off, seq_len, seq_func, seq_id=None):
        residues = np.ascontiguousarray(residues, dtype=np.uint8)
        seq_off = np.ascontiguousarray(seq_off, dtype=np.uint64)
        seq_len = np.ascontiguousarray(seq_len, dtype=np.uint32)
        seq_func = np.ascontiguousarray(seq_func, dtype=np.uint16)
        n = len(seq_len)
        assert len(seq_off) == n and len(seq_func) == n
        if n:
            end = seq_off.astype(np.int64) + seq_len.astype(np.int64)
            if end.max() > len(residues):
                raise SkmError("seq_off/seq_len exceed the residue buffer")
        sid = None if seq_id is None else np.ascontiguousarray(seq_id, dtype=np.uint32)
        _check(lib().skm_build_add_batch(self._h, _ptr(residues), _ptr(seq_off), _ptr(seq_len), _ptr(seq_func),
                                         _ptr(sid) if sid is not None else None, n))

    def reserve(self, n_residues: int, n_seqs: int):
        """skm_build_reserve: capacity hint so the HBM residue buffer is allocated once (batches
        stream to HBM through two alternating pinned staging buffers as they are added)."""
        _check(lib().skm_build_reserve(self._h, int(n_residues), int(n_seqs)))

    def set_transport(self, transport: "GlooTransport"):
        """Join the ranks through a host transport (skm_build_set_transport) instead of RCCL."""
        self._transport = transport  # the callbacks must outlive the handle's runs
        _check(lib().skm_build_set_transport(self._h, transport.ptr))

    def set_comm(self, unique_id: bytes):
        """Join the RCCL communicator (collective over the world_size ranks)."""
        buf = (C.c_uint8 * 128).from_buffer_copy(bytes(unique_id))
        _check(lib().skm_build_set_comm(self._h, buf))

    def prepare(self):
        _check(lib().skm_build_prepare(self._h))

    def run(self):
        _check(lib().skm_build_run(self._h))

    def timings(self) -> dict:
        ms = (C.c_float * 15)()
        n = lib().skm_build_last_timings(self._h, ms, 15)
        names = ["extract_count", "scan", "extract_scatter", "bucket_process", "overflow", "chains", "stats", "total",
                 "exchange", "partition", "bucket_kernel", "big_groups", "chain_tail", "giant_start", "giant_end"]
        return {names[i]: float(ms[i]) for i in range(n)}

    def set_kernel_timing(self, enable: bool, only: str | None = None):
        """Event pairs around every kernel launch of the next runs (or only kernel `only`)."""
        _check(lib().skm_build_set_kernel_timing(self._h, 1 if enable else 0, only.encode() if only else None))

    def kernel_timings(self) -> dict:
        """{kernel name: (total device ms, launches)} of the last run (set_kernel_timing)."""
        n = lib().skm_build_kernel_timings(self._h, None, 0, None, None, 0)
        if n <= 0:
            return {}
        ms = (C.c_float * n)()
        cnt = (C.c_uint64 * n)()
        buf = C.create_string_buffer(64 * n + 64)
        lib().skm_build_kernel_timings(self._h, buf, len(buf), ms, cnt, n)
        names = buf.value.decode().split("\n")[:n]
        return {names[i]: (float(ms[i]), int(cnt[i])) for i in range(n)}

    def set_option(self, name: str, value: int):
        """skm_build_set_option: "key_range_passes" (0 = automatic), "device_memory_budget_mb",
        and the diagnostic tunables named in include/skm.h."""
        _check(lib().skm_build_set_option(self._h, name.encode(), int(value)))

    def passes(self) -> int:
        """Key-range passes of the last run (1 when the shard fits the work buffers)."""
        return self.counters()["passes"]

    def counters(self) -> dict:
        v = (C.c_uint64 * 46)()
        n = lib().skm_build_counters(self._h, v, 46)
        names = ["windows", "kept", "overflow_subbuckets", "chain_jobs", "chain_samples", "sequences", "grouped",
                 "overflow_elements", "overflow_kept", "big_groups", "big_kept", "passes", "valid", "giant_chains",
                 "giant_max", "redone", "cap_overflow_scratch", "cap_split", "cap_long_samples", "cap_long_jobs",
                 "demand_overflow_scratch", "demand_split", "demand_long_samples", "demand_long_jobs",
                 "long_samples", "routed", "add_batch_us", "prepare_upload_us", "prepare_plan_us", "prepare_rest_us",
                 "pass_groups", "add_pack_us", "add_dma_wait_us", "finish_us", "finish_wait_us", "finish_copy_us",
                 "finish_chunks", "finish_select_dev_us", "finish_sort_dev_us", "finish_gather_dev_us",
                 "finish_d2h_dev_us", "finish_max_chunk", "finish_wide_index", "kept_cap",
                 "free_after_prepare", "recs_rot"]
        return {names[i]: int(v[i]) for i in range(n)}

    def debug_jobs(self, k: int = 64) -> list:
        v = (C.c_uint32 * k)()
        _check(lib().skm_build_debug_jobs(self._h, v, k))
        return [int(x) for x in v]

    def debug_overflow(self, k: int = 4096) -> list:
        """Element counts of the last pass's overflow sub-buckets, largest first."""
        v = (C.c_uint32 * k)()
        n = lib().skm_build_debug_overflow(self._h, v, k)
        return [int(x) for x in v[:min(max(n, 0), k)]]

    def debug_stamps(self, enable: bool) -> list:
        v = (C.c_uint64 * 32)()
        _check(lib().skm_build_debug_stamps(self._h, 1 if enable else 0, v, 32))
        return [int(x) for x in v]

    def finish(self) -> KeptKmers:
        k = _Kept()
        _check(lib().skm_build_finish(self._h, C.byref(k)))
        return self._kept(k)

    def finish_slice(self, slice_bits: int, slice_: int) -> KeptKmers:
        """skm_build_finish_slice: the kept k-mers whose slice hash (fmix64 of the key, top
        slice_bits bits) is slice_, keys sorted; statistics are the whole build's."""
        k = _Kept()
        _check(lib().skm_build_finish_slice(self._h, int(slice_bits), int(slice_), C.byref(k)))
        return self._kept(k)

    def signature_flags(self) -> np.ndarray:
        """Per-sequence signature flags of the last run (sequences with a kept function, add order)."""
        n = self.counters()["sequences"]
        out = np.zeros(max(n, 1), np.uint8)
        _check(lib().skm_build_signature_flags(self._h, _ptr(out), n))
        return out[:n]

    @staticmethod
    def _kept(k) -> KeptKmers:
        """The library's arrays without a copy: keys / data view the hand-off's host arrays, which
        skm_kept_free releases when the last view is gone."""
        owner = _KeptOwner(k)
        n = int(k.n)
        if n:
            kb = (C.c_char * (8 * n)).from_address(C.cast(k.keys, C.c_void_p).value)
            db = (C.c_char * (10 * n)).from_address(C.cast(k.data, C.c_void_p).value)
            kb._owner = db._owner = owner
            keys = np.frombuffer(kb, np.uint64)
            data = np.frombuffer(db, STORED_DTYPE)
        else:
            keys, data = np.zeros(0, np.uint64), np.zeros(0, STORED_DTYPE)
        nf = int(k.n_functions)
        df = np.ctypeslib.as_array(k.distinct_functions, shape=(max(nf, 1),))[:nf].copy()
        sw = np.ctypeslib.as_array(k.seqs_with_func, shape=(max(nf, 1),))[:nf].copy()
        return KeptKmers(keys, data, df, sw, int(k.n_seqs_with_signature), int(k.distinct_signatures),
                         int(k.n_windows))

    def close(self):
        if self._h:
            lib().skm_build_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class GlooTransport:
    """skm_transport over torch.distributed (the default process group, e.g. gloo on the host):
    the rank collectives of a multi-process build without RCCL (tests; CPU-side channels).
    Callbacks run on the calling thread; an exception is reported as a failed collective."""

    def __init__(self):
        import torch.distributed as dist
        self.dist = dist
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        self._cbs = (_A2A_T(self._a2a), _RED_T(self._red), _AGV_T(self._agv))
        self.struct = _Transport(None, *self._cbs)
        self.ptr = C.pointer(self.struct)

    @staticmethod
    def _buf(addr, n):
        import torch
        if n == 0:
            return torch.zeros(0, dtype=torch.uint8)
        return torch.frombuffer((C.c_uint8 * n).from_address(addr), dtype=torch.uint8)

    def _a2a(self, ctx, send, scnt, soff, recv, rcnt, roff):
        try:
            W, me = self.world, self.rank
            sc = [int(scnt[i]) for i in range(W)]
            so = [int(soff[i]) for i in range(W)]
            rc = [int(rcnt[i]) for i in range(W)]
            ro = [int(roff[i]) for i in range(W)]
            if sc[me]:
                C.memmove(recv + ro[me], send + so[me], sc[me])
            reqs = []
            for q in range(W):
                if q == me:
                    continue
                if sc[q]:
                    reqs.append(self.dist.isend(self._buf(send + so[q], sc[q]).clone(), q))
                if rc[q]:
                    reqs.append(self.dist.irecv(self._buf(recv + ro[q], rc[q]), q))
            for r in reqs:
                r.wait()
            return 0
        except Exception:  # reported to the library as a failed collective
            import traceback
            traceback.print_exc()
            return -1

    def _red(self, ctx, data, count, op):
        try:
            import torch
            n = int(count)
            if op == 0:
                a = np.ctypeslib.as_array(C.cast(data, C.POINTER(C.c_uint32)), shape=(n,))
                t = torch.from_numpy(a.astype(np.int64))
                self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
                a[:] = (t.numpy() & 0xFFFFFFFF).astype(np.uint32)
            else:
                a = np.ctypeslib.as_array(C.cast(data, C.POINTER(C.c_uint8)), shape=(n,))
                t = torch.from_numpy(a.astype(np.int32))
                self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
                a[:] = t.numpy().astype(np.uint8)
            return 0
        except Exception:
            import traceback
            traceback.print_exc()
            return -1

    def _agv(self, ctx, send, recv, bytes_per_rank):
        try:
            import torch
            W = self.world
            nb = [int(bytes_per_rank[i]) for i in range(W)]
            m = max(1, max(nb))
            mine = torch.zeros(m, dtype=torch.uint8)
            if nb[self.rank]:
                mine[:nb[self.rank]] = self._buf(send, nb[self.rank])
            outs = [torch.zeros(m, dtype=torch.uint8) for _ in range(W)]
            self.dist.all_gather(outs, mine)
            o = 0
            for r in range(W):
                if nb[r]:
                    self._buf(recv + o, nb[r])[:] = outs[r][:nb[r]]
                o += nb[r]
            return 0
        except Exception:
            import traceback
            traceback.print_exc()
            return -1


def comm_unique_id() -> bytes:
    """128-byte RCCL unique id (rank 0 creates it; broadcast it to every rank's set_comm)."""
    buf = (C.c_uint8 * 128)()
    _check(lib().skm_comm_unique_id(buf))
    return bytes(buf)


def group_run(builders) -> None:
    """Run ranks 0..n-1 of one build inside this process (device-copy exchange instead of RCCL);
    used to test the multi-GPU path on one device."""
    arr = (C.c_void_p * len(builders))(*[b._h.value for b in builders])
    _check(lib().skm_build_group_run(arr, len(builders)))


def mph_build(keys: np.ndarray, data: np.ndarray, mph_path: str, dat_path: str, seed: int = 1,
              device: int | None = None):
    """build_perfect_hash (perfect_hash.h:11-69): cmph-compatible BDZ .mph + dense .dat.
    device=None: host construction; device=d: parallel peeling on GPU d."""
    keys = np.ascontiguousarray(keys, dtype=np.uint64)
    data = np.ascontiguousarray(data, dtype=STORED_DTYPE)
    if device is None:
        _check(lib().skm_mph_build(_ptr(keys), _ptr(data), len(keys), seed, mph_path.encode(), dat_path.encode()))
    else:
        _check(lib().skm_mph_build_device(_ptr(keys), _ptr(data), len(keys), seed, mph_path.encode(),
                                          dat_path.encode(), device))


class _MphStats(C.Structure):
    _fields_ = [(n, C.c_double) for n in ("upload_s", "peel_s", "assign_s", "rank_s", "place_s", "verify_s",
                                          "write_s", "total_s")] + \
               [("n_keys", C.c_uint64), ("n_vertices", C.c_uint64), ("attempts", C.c_uint32),
                ("peel_rounds", C.c_uint32), ("verified", C.c_int32), ("pad", C.c_int32)]


def mph_build_device(keys: np.ndarray, data: np.ndarray, mph_path: str | None = None, dat_path: str | None = None,
                     seed: int = 1, device: int = 0, verify: bool = True) -> dict:
    """skm_mph_build_device_ex: the device BDZ construction (perfect_hash.h:11-69) up to cmph's
    32-bit vertex space, with its phase times; None paths skip writing that image; verify checks
    on the device that the slots are a permutation, that the annotate kernels' pair-line search
    agrees with bdz_search for every key and that every .dat record is its key's."""
    keys = np.ascontiguousarray(keys, dtype=np.uint64)
    data = np.ascontiguousarray(data, dtype=STORED_DTYPE)
    st = _MphStats()
    _check(lib().skm_mph_build_device_ex(_ptr(keys), _ptr(data), len(keys), seed,
                                         mph_path.encode() if mph_path else None,
                                         dat_path.encode() if dat_path else None, device, 1 if verify else 0,
                                         C.byref(st)))
    return {n: getattr(st, n) for n, _ in _MphStats._fields_ if n != "pad"}


class CmphKmerDb:
    """CmphKmerDb<StoredKmerData, 8> (cmph_kmer.h:28-164) resident in HBM."""
    KmerSize = K

    def __init__(self, file_base: str | None = None, device: int = 0, mph: bytes | None = None,
                 dat: bytes | None = None):
        self._h = C.c_void_p()
        self.device = device
        if file_base is not None:
            _check(lib().skm_db_open(C.byref(self._h), (file_base + ".mph").encode(), (file_base + ".dat").encode(),
                                     device))
        else:
            mb = np.frombuffer(mph, dtype=np.uint8)
            db = np.frombuffer(dat, dtype=np.uint8) if dat else np.zeros(0, np.uint8)
            _check(lib().skm_db_open_mem(C.byref(self._h), _ptr(mb), len(mb), _ptr(db), len(db), device))

    def hash_size(self) -> int:
        m = C.c_uint32()
        _check(lib().skm_db_size(self._h, C.byref(m)))
        return m.value

    def lookup_keys(self, keys: np.ndarray) -> np.ndarray:
        """cmph_search per key (lookup_key, cmph_kmer.h:90-92); >= hash_size means miss."""
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        out = np.zeros(len(keys), dtype=np.uint32)
        if len(keys):
            _check(lib().skm_db_lookup(self._h, _ptr(keys), len(keys), _ptr(out)))
        return out

    def lookup_keys_generic(self, keys: np.ndarray) -> np.ndarray:
        """Test hook: the generic bdz_search walk (skm_debug_db_lookup_generic), bypassing the
        b == 7 (g word, rank) pair lines that lookup_keys and the annotate kernels use."""
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        out = np.zeros(len(keys), dtype=np.uint32)
        if len(keys):
            _check(lib().skm_debug_db_lookup_generic(self._h, _ptr(keys), len(keys), _ptr(out)))
        return out

    def close(self):
        if self._h:
            lib().skm_db_close(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class KeptKmerDb(CmphKmerDb):
    """KeptKmerDB<8> (kept_kmer_db.h:9-31): exact-key DB over a build's kept k-mers, resident in HBM
    (the recall pass's DB, kmers-build-signatures.cc:238).  lookup_keys returns the record index
    of each key, len(keys) for a miss."""

    def __init__(self, keys: np.ndarray, data: np.ndarray, device: int = 0):
        self._h = C.c_void_p()
        self.device = device
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        data = np.ascontiguousarray(data, dtype=STORED_DTYPE)
        _check(lib().skm_db_open_kept(C.byref(self._h), _ptr(keys), _ptr(data), len(keys), device))


def read_function_index(path: str) -> list:
    """FunctionCaller::read_function_index (call_functions.tcc:123-148): column 1 by id."""
    rows = []
    with open(path, "rb") as f:
        for line in f.read().split(b"\n"):
            if not line:
                continue
            parts = line.split(b"\t")
            rows.append((int(parts[0]), parts[1].decode("latin-1") if len(parts) > 1 else ""))
    n = max((i for i, _ in rows), default=-1) + 1
    out = [""] * n
    for i, s in rows:
        out[i] = s
    return out


class QueryBatch:
    """A batch of query sequences resident in HBM (skm_query_*): run() repeats the device pipeline
    (window lookup + HitSet calls) without re-uploading; timings() = the last run's device ms."""

    def __init__(self, db: CmphKmerDb, residues, seq_off, seq_len):
        self._h = C.c_void_p()
        self.db = db
        residues = np.ascontiguousarray(residues, dtype=np.uint8)
        seq_off = np.ascontiguousarray(seq_off, dtype=np.uint64)
        seq_len = np.ascontiguousarray(seq_len, dtype=np.uint32)
        self._n_seqs = len(seq_len)
        _check(lib().skm_query_create(C.byref(self._h), db._h, _ptr(residues), _ptr(seq_off), _ptr(seq_len),
                                      len(seq_len)))

    def run(self, hypo_index: int, ignore_hypo: bool = False, min_hits: int = 5, max_gap: int = 200):
        opts = _AnnotOpts(min_hits, max_gap, int(ignore_hypo), hypo_index, 0, 0)
        _check(lib().skm_query_run(self._h, C.byref(opts)))

    def timings(self) -> dict:
        ms = (C.c_float * 4)()
        n = lib().skm_query_last_timings(self._h, ms, 4)
        return dict(zip(["lookup", "hitset", "compact", "total"], list(ms)[:n]))

    def calls(self):
        out = _Calls()
        _check(lib().skm_query_calls(self._h, C.byref(out)))
        try:
            n, nc = int(out.n_seqs), int(out.n_calls)
            off = np.ctypeslib.as_array(out.call_off, shape=(n + 1,)).copy()
            calls = (np.frombuffer(C.string_at(out.calls, CALL_DTYPE.itemsize * nc), dtype=CALL_DTYPE).copy()
                     if nc else np.zeros(0, CALL_DTYPE))
            return off, calls
        finally:
            lib().skm_calls_free(C.byref(out))

    def window_hits(self):
        """skm_query_window_hits: (hit_off [n+1], pos, fm) of the last run -- every window the
        device lookup found in the DB, as (offset in its sequence, function_index << 16 | mean)."""
        n_seqs = self._n_seqs
        off = np.zeros(n_seqs + 1, np.uint64)
        n = C.c_uint64(0)
        _check(lib().skm_query_window_hits(self._h, _ptr(off), None, None, 0, C.byref(n)))
        pos = np.zeros(max(int(n.value), 1), np.uint32)
        fm = np.zeros(max(int(n.value), 1), np.uint32)
        _check(lib().skm_query_window_hits(self._h, _ptr(off), _ptr(pos), _ptr(fm), len(pos), C.byref(n)))
        return off, pos[:n.value], fm[:n.value]

    def close(self):
        if self._h:
            lib().skm_query_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class FunctionCaller:
    """FunctionCaller<CmphKmerDb> (call_functions.h:60-136) with the per-window lookup and HitSet
    state machine on the GPU and find_best_call on the host."""

    def __init__(self, db: CmphKmerDb, function_index, min_hits: int = 5, max_gap: int = 200,
                 mean_mode: int = 0, mad_mode: int = 0):
        """mean_mode / mad_mode: the Boost.Math the reference was compiled against
        (call_functions.tcc:51-53): 0 / 0 = >= 1.76 (four-lane mean, |x(mid) - median| MAD),
        1 / 1 = the older single running mean and the MAD that returns |x(mid)|."""
        self.db = db
        self.function_index = read_function_index(function_index) if isinstance(function_index, str) \
            else list(function_index)
        self.min_hits = min_hits
        self.max_gap = max_gap
        self.ignore_hypothetical_ = False
        self.mean_mode = mean_mode
        self.mad_mode = mad_mode
        try:
            self.hypo_index = self.function_index.index("hypothetical protein")
        except ValueError:
            self.hypo_index = -1
        self._fi_arr = _fi_array(self.function_index)

    def ignore_hypothetical(self, x: bool):
        self.ignore_hypothetical_ = bool(x)

    def _opts(self):
        return _AnnotOpts(self.min_hits, self.max_gap, 1 if self.ignore_hypothetical_ else 0, self.hypo_index,
                          self.mean_mode, self.mad_mode)

    def process_seqs(self, residues, seq_off, seq_len):
        """process_aa_seq for a batch: returns (call_off u64[n+1], calls CALL_DTYPE)."""
        if self.hypo_index < 0:  # call_functions.tcc:269-274 exits the process
            raise SkmError("Cannot find hypothetical protein index")
        residues = np.ascontiguousarray(residues, dtype=np.uint8)
        seq_off = np.ascontiguousarray(seq_off, dtype=np.uint64)
        seq_len = np.ascontiguousarray(seq_len, dtype=np.uint32)
        out = _Calls()
        opts = self._opts()
        _check(lib().skm_annotate(self.db._h, _ptr(residues), _ptr(seq_off), _ptr(seq_len), len(seq_len),
                                  C.byref(opts), C.byref(out)))
        try:
            n = int(out.n_seqs)
            off = np.ctypeslib.as_array(out.call_off, shape=(n + 1,)).copy()
            nc = int(out.n_calls)
            calls = (np.frombuffer(C.string_at(out.calls, CALL_DTYPE.itemsize * nc), dtype=CALL_DTYPE).copy()
                     if nc else np.zeros(0, CALL_DTYPE))
            return off, calls
        finally:
            lib().skm_calls_free(C.byref(out))

    def find_best_call(self, calls: np.ndarray):
        """find_best_call (call_functions.tcc:347-659) -> (function_index, function, score, offset)."""
        return _find_best_call(calls, self._fi_arr, len(self.function_index))


def _fi_array(function_index):
    return (C.c_char_p * max(1, len(function_index)))(*[s.encode("latin-1") for s in function_index])


def _find_best_call(calls, fi_arr, nfunc):
    calls = np.ascontiguousarray(calls, dtype=CALL_DTYPE)
    fi = C.c_uint16()
    score = C.c_float()
    off = C.c_float()
    buf = C.create_string_buffer(4096)
    _check(lib().skm_find_best_call(_ptr(calls) if len(calls) else None, len(calls), fi_arr, nfunc, C.byref(fi),
                                    C.byref(score), C.byref(off), buf, 4096))
    return fi.value, buf.value.decode("latin-1"), score.value, off.value


def find_best_call(calls: np.ndarray, function_index):
    """Host find_best_call (call_functions.tcc:347-659) over one sequence's calls, without a DB:
    -> (function_index, function, score, offset)."""
    return _find_best_call(calls, _fi_array(function_index), len(function_index))


class SeqIdMap:
    """SeqIdMap (seq_id_map.h:7-35): id -> index in order of first appearance."""

    def __init__(self):
        self._index = {}
        self._ids = []

    def lookup_id(self, id_: str) -> int:
        i = self._index.get(id_)
        if i is None:
            i = len(self._ids)
            self._index[id_] = i
            self._ids.append(id_)
        return i

    def lookup_index(self, i: int) -> str:
        return self._ids[i]

    def __len__(self):
        return len(self._ids)


def matrix_tile_rows(n_idx: int, rank: int, world: int):
    """Row band [begin, end) of GPU `rank` of `world` with (nearly) equal upper-triangle area."""
    a, b = C.c_uint32(), C.c_uint32()
    _check(lib().skm_matrix_tile_rows(n_idx, rank, world, C.byref(a), C.byref(b)))
    return a.value, b.value


class MatrixDistance:
    """MatrixDistance<FunctionCaller<CmphKmerDb>> (matrix_distance.h:30-179) / kmers-matrix-distance
    (kmers-matrix-distance.cc:94-212): shared-signature-k-mer counts over every pair of query
    sequences, on the GPU (skm_matrix_*).  seq_idx: SeqIdMap index per sequence (default: 0..n-1);
    rows=(begin, end) restricts the counts to pairs whose first index lies in [begin, end) -- one
    GPU's tile (matrix_tile_rows)."""

    def __init__(self, db: CmphKmerDb, function_index, residues, seq_off, seq_len, seq_idx=None,
                 n_idx: int | None = None):
        self.db = db
        fi = read_function_index(function_index) if isinstance(function_index, str) else list(function_index)
        if "hypothetical protein" not in fi:  # call_functions.tcc:269-274 exits the process
            raise SkmError("Cannot find hypothetical protein index")
        self.hypo_index = fi.index("hypothetical protein")
        residues = np.ascontiguousarray(residues, dtype=np.uint8)
        seq_off = np.ascontiguousarray(seq_off, dtype=np.uint64)
        seq_len = np.ascontiguousarray(seq_len, dtype=np.uint32)
        if seq_idx is None:
            seq_idx = np.arange(len(seq_len), dtype=np.uint32)
        seq_idx = np.ascontiguousarray(seq_idx, dtype=np.uint32)
        self.n_idx = int(n_idx if n_idx is not None else (int(seq_idx.max()) + 1 if len(seq_idx) else 0))
        self._h = C.c_void_p()
        _check(lib().skm_matrix_create(C.byref(self._h), db._h, _ptr(residues), _ptr(seq_off), _ptr(seq_len),
                                       _ptr(seq_idx), len(seq_len), self.n_idx))

    def set_transport(self, transport: "GlooTransport"):
        """Join the ranks of a multi-GPU matrix distance through a host transport: this handle's
        queries are rank transport.rank's range; run() becomes collective and pairs() returns the
        rank's row band (skm_matrix_tile_rows)."""
        self._transport = transport
        _check(lib().skm_matrix_set_transport(self._h, transport.rank, transport.world, transport.ptr))

    def set_comm(self, unique_id: bytes, rank: int, world: int):
        """Join the ranks over RCCL (collective; rank 0's comm_unique_id broadcast to every rank)."""
        buf = (C.c_uint8 * 128).from_buffer_copy(bytes(unique_id))
        _check(lib().skm_matrix_set_comm(self._h, rank, world, buf))

    def run(self, rows=None, max_tile_bytes: int = 0):
        a, b = rows if rows is not None else (0, 0)
        opts = _MatrixOpts(self.hypo_index, a, b, 0, max_tile_bytes)
        _check(lib().skm_matrix_run(self._h, C.byref(opts)))

    def timings(self) -> dict:
        ms = (C.c_float * 5)()
        n = lib().skm_matrix_last_timings(self._h, ms, 5)
        return dict(zip(["hits", "group", "pairs", "emit", "total"], list(ms)[:n]))

    def counters(self) -> dict:
        v = (C.c_uint64 * 7)()
        n = lib().skm_matrix_counters(self._h, v, 7)
        return dict(zip(["windows", "hits", "increments", "pairs", "kmers", "local_hits", "routed"],
                        [int(x) for x in list(v)[:n]]))

    def pairs(self) -> np.ndarray:
        """(n, 3) u32 (id1, id2, count), id1 < id2, sorted by (id1, id2)."""
        out = _Pairs()
        _check(lib().skm_matrix_pairs(self._h, C.byref(out)))
        try:
            n = int(out.n)
            if n == 0:
                return np.zeros((0, 3), np.uint32)
            return np.ctypeslib.as_array(out.pairs, shape=(n * 3,)).reshape(n, 3).copy()
        finally:
            lib().skm_pairs_free(C.byref(out))

    def compute(self, rows=None):
        self.run(rows)
        return self.pairs()

    def close(self):
        if self._h:
            lib().skm_matrix_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
