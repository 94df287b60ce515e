"""The slice-restricted oracle (oracle_build_sel_mt, the checker of the 50M-protein C3 build in
tests/test_gpu_c3.py) on the CPU: the 2^b slices of the key space -- fmix64(key) top b bits, the
same public hash skm_build_finish_slice selects with -- partition the single-thread oracle's
kept set, each slice bit for bit, and their signature flags OR to the full build's."""
import numpy as np
import pytest

import oracle_ref
from signature_kmers_amd import synth


@pytest.mark.parametrize("bits", [1, 3])
def test_slices_partition_the_oracle_build(bits):
    p = synth.generate_arrays(6000, 60, per_file=1000, seed=3)
    r, o, l, f, i, funcs = synth.build_inputs(p)
    ref = oracle_ref.build(r, o, l, f, i, len(funcs))
    h = oracle_ref.slice_hash(ref["keys"]) >> np.uint64(64 - bits)
    full = oracle_ref.build_slice_mt(r, o, l, f, i, len(funcs), 4, 0, 0, want_flags=True)
    assert np.array_equal(full["keys"], ref["keys"])
    assert full["n_seqs_with_signature"] == ref["n_seqs_with_signature"] == int(full["flags"].sum())
    total, flags = 0, np.zeros_like(full["flags"])
    for s in range(1 << bits):
        got = oracle_ref.build_slice_mt(r, o, l, f, i, len(funcs), 4, bits, s, want_flags=True)
        m = h == s
        assert np.array_equal(got["keys"], ref["keys"][m])
        assert np.array_equal(got["data"].view(np.uint8), ref["data"][m].view(np.uint8))
        assert np.array_equal(got["distinct_functions"],
                              np.bincount(ref["data"]["function_index"][m], minlength=len(funcs))[:len(funcs)])
        assert got["valid_windows"] == full["valid_windows"]
        total += len(got["keys"])
        flags |= got["flags"]
    assert total == len(ref["keys"])
    assert np.array_equal(flags, full["flags"])


def test_slice_hash_is_murmur3_fmix64():
    # fmix64 known values: fmix64(0) = 0, and the finalizer is a bijection on 64-bit words
    assert int(oracle_ref.slice_hash(np.array([0], np.uint64))[0]) == 0
    x = np.arange(1, 100001, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
    assert len(np.unique(oracle_ref.slice_hash(x))) == len(x)
