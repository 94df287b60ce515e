"""Parity at the headline size: the 50M-protein C3 proteome (BASELINE configs[2], the bench's
headline workload) built on ONE GPU with its key-range passes, checked against the oracle.

The whole C3 build (15.2 G windows, ~2.9 G kept k-mers) cannot be restated on the host in the
reference's way (~780 GB for the multimap), so the check is split:

* bit-exact on one output slice: the kept k-mers whose fmix64(key) has top 6 bits == SLICE
  (skm_build_finish_slice) against oracle_build_sel_mt, which groups only the windows of those
  keys -- every key's occurrences are all in or all out, so each selected group is exactly the
  reference's group (signature_build.tcc:184-293).  The slice is 1/64 of the key space and holds
  k-mers with >= 2^14 occurrences (asserted), i.e. the heavy-key split, the overflow path and the
  stashed long P^2 chains at their C3 depths;
* size-independent properties over the whole build: the occurrences grouped equal the oracle's
  count of valid windows of the whole input (every window extracted once, none lost by the
  key-range passes or the per-pass compaction), seqs_with_func equals the per-function sequence
  count, distinct_signatures == kept == sum(distinct_functions), num_seqs_with_a_signature equals
  the device's per-sequence flags and every sequence the oracle flags for the slice is flagged.
The generator is the bench's (seed 20241115, 12,500 files of 4,000 proteins)."""
import os

import numpy as np
import pytest

import oracle_ref
from signature_kmers_amd import synth

pytestmark = pytest.mark.gpu

N_C3, FAM, PER_FILE = 50_000_000, 4000, 4000
SLICE_BITS, SLICE = 6, 0


def _threads():
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            return max(1, min(len(os.sched_getaffinity(0)), int(q) // int(p)))
    except (OSError, ValueError):
        pass
    return len(os.sched_getaffinity(0))


def test_c3_slice_bit_exact_and_whole_build_properties(skm, gpu):
    T = _threads()
    parts = list(synth.iter_file_inputs(N_C3, FAM, PER_FILE, workers=min(16, T)))
    funcs = synth.functions(FAM)
    nf = len(funcs)
    b = skm.SignatureBuilder(nf)
    b.reserve(sum(len(p[0]) for p in parts), sum(len(p[2]) for p in parts))
    for r, o, l, f, i in parts:
        b.add_batch(r, o, l, f, i)
    b.run()
    c = b.counters()
    got = b.finish_slice(SLICE_BITS, SLICE)
    flags = b.signature_flags()
    b.close()
    assert c["passes"] >= 8, c  # the headline's out-of-core path (16 passes at 288 GB)
    # pack the input for the oracle (16.5 GB of residues)
    lens = np.concatenate([p[2] for p in parts])
    func = np.concatenate([p[3] for p in parts])
    ids = np.concatenate([p[4] for p in parts])
    res = np.concatenate([p[0] for p in parts])
    del parts
    off = np.zeros(len(lens), np.uint64)
    off[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    ref = oracle_ref.build_slice_mt(res, off, lens, func, ids, nf, T, SLICE_BITS, SLICE, want_flags=True)
    # ---- the slice, bit for bit ----
    assert ref["max_group"] >= 1 << 14, ref["max_group"]  # heavy keys / long chains are in the slice
    assert len(got.keys) == len(ref["keys"]) > 10_000_000, (len(got.keys), len(ref["keys"]))
    assert np.array_equal(got.keys, ref["keys"])
    for fld in ("avg_from_end", "function_index", "mean", "median", "var"):
        bad = np.nonzero(got.data[fld] != ref["data"][fld])[0]
        assert len(bad) == 0, (fld, len(bad), got.keys[bad[:5]], got.data[bad[:5]], ref["data"][bad[:5]])
    assert np.array_equal(np.bincount(got.data["function_index"], minlength=nf)[:nf], ref["distinct_functions"])
    # ---- the whole build ----
    kept_fn = func != 0xFFFF
    assert c["windows"] == oracle_ref.count_windows(lens, func)
    assert c["grouped"] == c["valid"] == ref["valid_windows"], (c["grouped"], c["valid"], ref["valid_windows"])
    assert np.array_equal(got.seqs_with_func, np.bincount(func[kept_fn], minlength=nf)[:nf])
    assert got.distinct_signatures == c["kept"] == int(got.distinct_functions.astype(np.int64).sum())
    assert len(flags) == int(kept_fn.sum())
    assert got.n_seqs_with_signature == int(flags.sum()) <= len(flags)
    oflags = ref["flags"][kept_fn]
    assert int(oflags.sum()) > 0 and not np.any(oflags & ~flags), "a sequence with a kept slice k-mer is unflagged"
