"""GPU parity: HIP signature build (libskm via the C-ABI) vs the CPU oracle restatement.

Bit-exact comparison of the kept k-mer set, every StoredKmerData field, distinct_functions,
seqs_with_func, num_seqs_with_a_signature and distinct_signatures on seeded inputs."""
import numpy as np
import pytest

import oracle_ref
from signature_kmers_amd import synth

pytestmark = pytest.mark.gpu


def run_both(skm, residues, seq_off, seq_len, seq_func, seq_id, nf, options=None):
    b = skm.SignatureBuilder(nf)
    for k, v in (options or {}).items():
        b.set_option(k, v)
    b.add_batch(residues, seq_off, seq_len, seq_func, seq_id)
    got = b.finish()
    b.close()
    ref = oracle_ref.build(residues, seq_off, seq_len, seq_func, seq_id, nf)
    return got, ref


def assert_same(got, ref):
    assert len(got.keys) == len(ref["keys"]), (len(got.keys), len(ref["keys"]))
    np.testing.assert_array_equal(got.keys, ref["keys"])
    for f in ("avg_from_end", "function_index", "mean", "median", "var"):
        bad = np.nonzero(got.data[f] != ref["data"][f])[0]
        assert len(bad) == 0, (f, len(bad), got.data[bad[:5]], ref["data"][bad[:5]],
                               [skm_kmer(k) for k in got.keys[bad[:5]]])
    np.testing.assert_array_equal(got.distinct_functions, ref["distinct_functions"])
    np.testing.assert_array_equal(got.seqs_with_func, ref["seqs_with_func"])
    assert got.n_seqs_with_signature == ref["n_seqs_with_signature"]
    assert got.distinct_signatures == ref["distinct_signatures"]


def skm_kmer(k):
    return int(k).to_bytes(8, "little")


def pack(seqs):
    lens = np.array([len(s) for s in seqs], np.uint32)
    off = np.zeros(len(seqs), np.uint64)
    if len(seqs):
        off[1:] = np.cumsum(lens[:-1])
    res = np.frombuffer(b"".join(seqs), np.uint8) if seqs else np.zeros(0, np.uint8)
    return res, off, lens


def test_config1_synthetic(skm, gpu):
    p = synth.generate_arrays(1000, 40, per_file=100, extras=True)
    r, o, l, f, i, funcs = synth.build_inputs(p)
    got, ref = run_both(skm, r, o, l, f, i, len(funcs))
    assert len(got.keys) > 1000
    assert_same(got, ref)


@pytest.mark.parametrize("n,fam,seed", [(5000, 100, 1), (20000, 400, 2)])
def test_synthetic_sizes(skm, gpu, n, fam, seed):
    p = synth.generate_arrays(n, fam, per_file=1000, seed=seed)
    r, o, l, f, i, funcs = synth.build_inputs(p)
    got, ref = run_both(skm, r, o, l, f, i, len(funcs))
    assert_same(got, ref)


def test_level2_partition_and_overflow(skm, gpu):
    # 60K sequences from 60 families: level-1 buckets exceed LDS capacity (level-2 partition),
    # conserved k-mers of the largest families exceed a sub-bucket (global-memory overflow path)
    p = synth.generate_arrays(60000, 60, per_file=2000, seed=3)
    r, o, l, f, i, funcs = synth.build_inputs(p)
    got, ref = run_both(skm, r, o, l, f, i, len(funcs))
    assert_same(got, ref)


@pytest.mark.parametrize("inline_min", [16, 1000000000])
def test_overflow_inline_chains(skm, gpu, inline_min):
    # every overflow chain of >= 16 samples inline in k_overflow (wave-pair chain code, up to
    # OVF_INLINE_CAP per workgroup, the rest as jobs) -- and none inline
    p = synth.generate_arrays(60000, 60, per_file=2000, seed=4)
    r, o, l, f, i, funcs = synth.build_inputs(p)
    got, ref = run_both(skm, r, o, l, f, i, len(funcs), {"overflow_inline_min": inline_min})
    assert_same(got, ref)


@pytest.mark.parametrize("passes,long_class,opts", [(1, 6, {}), (2, 14, {}), (4, 8, {}), (64, 14, {}),
                                                   (4, 8, {"stage_round": 0}), (4, 8, {"partition_round": 1}),
                                                   (4, 8, {"partition_round": 2}), (1, 6, {"flag_check": 1, "flag_bits": 0}), (4, 8, {"flag_bits": 0}),
                                                   (4, 8, {"serial_overflow": 1}), (4, 8, {"chain_cus": 32}),
                                                   (4, 8, {"side_cus": 64}),
                                                   (4, 8, {"overlap": 1}), (16, 8, {"overlap": 1}),
                                                   (4, 8, {"overlap": 1, "serial_overflow": 1}),
                                                   (4, 8, {"lane_long": 0}), (16, 8, {"lane_long": 600}),
                                                   (16, 8, {"tail_defer": 1, "recs_rot": 1}), (4, 8, {"recs_rot": 1}),
                                                   (16, 8, {"big_split": 1, "emit_group": 16}),
                                                   (16, 8, {"part_order": 0}), (16, 8, {"part_split": 0})])
def test_key_range_passes(skm, gpu, passes, long_class, opts):
    """Out-of-core build: P passes over disjoint k-mer ranges (each k-mer in exactly one pass)
    give the single-pass result bit for bit, overflow sub-buckets and chains included, and a
    second run over the same handle repeats it (arena cursor, flags and counters reset).  Low
    long-chain classes send most chains through the stash + chain streams that outlive a pass.
    opts: the staging / partition round-size variants (stage_round 0: full rounds;
    partition_round 1, 2: rounds of 4096 with 512 / 1024 threads), flag_check, serial_overflow, chain_cus / side_cus (the long-chain / overflow
    and selection streams on a subset of the CUs), overlap 1 (pipelined passes: a second element
    buffer set, the pass's overflow path beside the next pass), lane_long 0 / 600 (every stashed long
    chain on a wave pair / the ones of >= 600 samples: the others one lane each, k_chains),
    tail_defer / recs_rot (the pass tail issued after the next pass's scan; the split alternating two
    element buffers), big_split with emit_group 16 (one residue scan for all 16 passes), part_order 0
    / part_split 0 (k_partition in bucket order / the oversized buckets not split off to stream 2)."""
    p = synth.generate_arrays(60000, 60, per_file=2000, seed=6)
    r, o, l, f, i, funcs = synth.build_inputs(p)
    ref = oracle_ref.build(r, o, l, f, i, len(funcs))
    b = skm.SignatureBuilder(len(funcs))
    b.set_option("key_range_passes", passes)
    for k, v in opts.items():
        b.set_option(k, v)
    b.set_option("main_long_class", long_class)
    b.set_option("overflow_long_class", long_class)
    b.add_batch(r, o, l, f, i)
    b.run()
    c1 = b.counters()
    b.run()
    assert b.counters() == c1
    got = b.finish()
    b.close()
    assert_same(got, ref)
    assert c1["overflow_subbuckets"] > 0 and c1["grouped"] == oracle_ref.count_windows(l, f) - _invalid(r, o, l, f)
    if opts.get("recs_rot") and passes > 1:
        assert c1["recs_rot"] == 1  # the second element buffer fits at this size


@pytest.mark.parametrize("passes,route_min,vacate", [(4, 256, 0), (16, 64, 0), (64, 1024, 0), (16, 64, 4), (16, 64, 1),
                                                     (4, 256, -1), (64, 1024, -1), (0, 256, -1)])
def test_heavy_key_routing(skm, gpu, passes, route_min, vacate):
    """Heavy-key routing (route_heavy_min): the k-mers whose sampled occurrence estimate reaches the
    threshold are grouped in the first half of the key-range passes, their elements carrying
    (natural pass ^ routed pass) above the rem bits so the key decodes back -- the kept set is the
    oracle's bit for bit, and many occurrences were actually routed.  vacate = -1: route_first, a
    heavy-only pass 0 (the light keys of pass 0 spread over the others; passes = 0 -> one pass by
    the budget, doubled to two)."""
    p = synth.generate_arrays(60000, 60, per_file=2000, seed=6)
    r, o, l, f, i, funcs = synth.build_inputs(p)
    ref = oracle_ref.build(r, o, l, f, i, len(funcs))
    b = skm.SignatureBuilder(len(funcs))
    b.set_option("key_range_passes", passes)
    b.set_option("route_heavy_min", route_min)
    if vacate >= 0:
        b.set_option("route_vacate", vacate)  # 0: the second half; else the last `vacate` passes, spread
    else:
        b.set_option("route_first", 1)
        b.set_option("route_first_min", route_min)
        b.set_option("giant_class", 8)  # the heavy pass's chains on the giant streams, timed
    b.set_option("main_long_class", 8)
    b.set_option("overflow_long_class", 8)
    b.add_batch(r, o, l, f, i)
    b.run()
    c = b.counters()
    t = b.timings()
    got = b.finish()
    b.close()
    assert c["routed"] > 100_000, c
    assert c["grouped"] == c["valid"]
    if vacate < 0:
        assert c["passes"] == (passes or 2) and c["giant_chains"] > 0, c
        assert 0 <= t["giant_start"] <= t["giant_end"] <= t["total"], t
    assert_same(got, ref)


@pytest.mark.parametrize("passes", [0, 4])
def test_work_buffers_grow_and_redo(skm, gpu, passes):
    """The data-sized work buffers (overflow scratch, split path, stashed long chains) start far
    too small: the step runs without a host round trip, records its demands on the device, and is
    redone with the buffers grown; the result is the oracle's bit for bit, and the next run on the
    same handle needs no redo.  With passes, every slot of the stashed long-job list starts as a
    canary job (poison_jobs): a long chain launched on a slot that no stash wrote -- the first,
    too-small attempt reserves none -- would overwrite the canary record and fail the run."""
    p = synth.generate_arrays(60000, 60, per_file=2000, seed=6)
    r, o, l, f, i, funcs = synth.build_inputs(p)
    ref = oracle_ref.build(r, o, l, f, i, len(funcs))
    b = skm.SignatureBuilder(len(funcs))
    if passes:
        b.set_option("key_range_passes", passes)
        b.set_option("poison_jobs", 1)
    b.set_option("main_long_class", 8)
    b.set_option("overflow_long_class", 8)
    b.set_option("work_buffer_elements", 64)
    b.add_batch(r, o, l, f, i)
    b.run()
    c1 = b.counters()
    assert c1["redone"] >= 1, c1
    assert c1["demand_overflow_scratch"] <= c1["cap_overflow_scratch"]
    assert c1["demand_split"] <= c1["cap_split"]
    if passes:
        assert 0 < c1["demand_long_samples"] <= c1["cap_long_samples"]
    b.run()
    assert b.counters()["redone"] == c1["redone"]
    got = b.finish()
    b.close()
    assert_same(got, ref)


def _invalid(r, o, l, f):
    ok = np.zeros(256, bool)
    ok[np.frombuffer(b"ACDEFGHIKLMNPQRSTVWYacdefghiklmnpqrstvwy", np.uint8)] = True
    good = ok[r].astype(np.int64)
    c = np.concatenate([[0], np.cumsum(good)])
    bad = 0
    for s0, ln, fn in zip(o.astype(np.int64), l.astype(np.int64), f):
        if fn == 0xFFFF or ln < 8:
            continue
        bad += int(((c[s0 + 8:s0 + ln + 1] - c[s0:s0 + ln - 7]) != 8).sum())
    return bad


def test_automatic_passes_from_memory_budget(skm, gpu):
    """A device-memory budget too small for one pass makes the build plan several passes by
    itself (the 50M-proteome path on one GPU), with the same result."""
    p = synth.generate_arrays(20000, 40, per_file=1000, seed=7)
    r, o, l, f, i, funcs = synth.build_inputs(p)
    got, ref = run_both(skm, r, o, l, f, i, len(funcs), {"device_memory_budget_mb": 600})
    assert_same(got, ref)


def test_edge_cases(skm, gpu):
    seqs = [
        b"",                       # empty
        b"ACDEFGH",                # 7 residues: no window
        b"ACDEFGHI",               # exactly one window
        b"ACDEFGHIXKLMNPQRST",     # X splits windows
        b"acdefghiklmnpqrstvwy",   # lower case is valid for the build
        b"ACDEFGHIBZUJOACDEFGHI",  # B/Z/U/J/O are not in ok_prot_
        b"ACDEFGHI*",              # '*' invalid
        b"WWWWWWWWWWWWWWWWWWWWWWWW",  # self-overlapping repeats
    ]
    res, off, lens = pack(seqs)
    func = np.array([0, 1, 2, 3, 4, 5, 0xFFFF, 2], np.uint16)
    sid = np.arange(len(seqs), dtype=np.uint32)
    got, ref = run_both(skm, res, off, lens, func, sid, 8)
    assert_same(got, ref)


def test_empty_input(skm, gpu):
    res, off, lens = pack([])
    got, ref = run_both(skm, res, off, lens, np.zeros(0, np.uint16), np.zeros(0, np.uint32), 4)
    assert len(got.keys) == 0 and got.distinct_signatures == 0
    assert_same(got, ref)


def test_cut_ties_and_heavy_groups(skm, gpu):
    rng = np.random.default_rng(5)
    core = bytes(rng.choice(np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY", np.uint8), 40))
    seqs, funcs = [], []
    # 4 copies func 3, 1 copy func 1  -> count 5, best 4 >= 4.0 -> kept with func 3
    # 5 copies func 2, 5 copies func 0 -> tie -> lowest index 0, 5 < 8 -> cut
    # 9000 copies func 1 (varying lengths) -> heavy group beyond LDS capacity
    for _ in range(4):
        seqs.append(b"MK" + core)
        funcs.append(3)
    seqs.append(b"MK" + core + b"G")
    funcs.append(1)
    tie = bytes(rng.choice(np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY", np.uint8), 30))
    for j in range(10):
        seqs.append(tie + b"A" * j)
        funcs.append(2 if j < 5 else 0)
    heavy = bytes(rng.choice(np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY", np.uint8), 25))
    for j in range(9000):
        pad = bytes(rng.choice(np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY", np.uint8), int(rng.integers(0, 300))))
        seqs.append(pad + heavy + pad[::-1])
        funcs.append(1 if j % 10 else 4)
    res, off, lens = pack(seqs)
    func = np.array(funcs, np.uint16)
    sid = np.arange(len(seqs), dtype=np.uint32)
    got, ref = run_both(skm, res, off, lens, func, sid, 6)
    assert_same(got, ref)


def test_u16_wrap_long_protein(skm, gpu):
    # protein longer than 65535: offsets wrap (signature_build.tcc:164), sums wrap in the mean
    rng = np.random.default_rng(9)
    aa = np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY", np.uint8)
    long = bytes(rng.choice(aa, 70000))
    seqs = [long, long[:30000], long[1000:1400]] + [long[5000:5300]] * 300
    res, off, lens = pack(seqs)
    func = np.zeros(len(seqs), np.uint16)
    sid = np.arange(len(seqs), dtype=np.uint32)
    got, ref = run_both(skm, res, off, lens, func, sid, 2)
    assert_same(got, ref)


def test_colliding_seq_ids(skm, gpu):
    p = synth.generate_arrays(3000, 30, per_file=1000, seed=11)
    r, o, l, f, i, funcs = synth.build_inputs(p)
    i = (i % 700).astype(np.uint32)  # many sequences share ids (files with > max_seqs_per_file)
    got, ref = run_both(skm, r, o, l, f, i, len(funcs))
    assert_same(got, ref)


def test_rerun_is_idempotent(skm, gpu):
    p = synth.generate_arrays(2000, 50, per_file=500, seed=4)
    r, o, l, f, i, funcs = synth.build_inputs(p)
    b = skm.SignatureBuilder(len(funcs))
    b.add_batch(r, o, l, f, i)
    b.run()
    a = b.finish()
    b.run()
    c = b.finish()
    np.testing.assert_array_equal(a.keys, c.keys)
    np.testing.assert_array_equal(a.data, c.data)


def test_handoff_wide_index_and_small_chunks(skm, gpu):
    """The finish hand-off's u64-index form (used from 2^32 kept k-mers, e.g. rank 0's gathered set
    of a multi-GPU build) and memory-capped small chunks give the same sorted kept set."""
    p = synth.generate_arrays(20000, 400, per_file=500, seed=8)
    r, o, l, f, i, funcs = synth.build_inputs(p)
    b = skm.SignatureBuilder(len(funcs))
    b.add_batch(r, o, l, f, i)
    a = b.finish()
    assert b.counters()["finish_wide_index"] == 0
    b.set_option("handoff_index_limit", 1)
    b.set_option("handoff_max_chunk", 1 << 14)
    c = b.finish()
    k = b.counters()
    b.close()
    assert k["finish_wide_index"] == 1 and k["finish_chunks"] > 4 and len(a.keys) > 1 << 16
    np.testing.assert_array_equal(a.keys, c.keys)
    np.testing.assert_array_equal(a.data.view(np.uint8), c.data.view(np.uint8))
    ref = oracle_ref.build(r, o, l, f, i, len(funcs))
    assert_same(c, ref)


def test_device_exact_division(skm, gpu):
    # reciprocal of every integer up to 2^22 (both signs) and 2^22 * 64 random quotients
    assert skm.debug_div_check(1 << 22, 64) == 0


@pytest.mark.parametrize("passes,giant_class,clustered,lsd", [(0, 0, False, 0), (0, 11, False, 0), (2, 12, False, 0),
                                                           (4, 17, False, 0), (0, 0, True, 0), (4, 17, True, 0),
                                                           (0, 0, False, 1), (2, 12, True, 1)])
def test_heavy_keys_split_path(skm, gpu, passes, giant_class, clustered, lsd):
    """k_ovf_split / k_heavy: overflow sub-buckets of >= 4096 elements lose their keys of >= 1024
    occurrences to the heavy path: one read for the per-function counts (LDS table: the exact best
    function for the fp32 80 % cut), the offset's high byte and the members per sequence-index
    bucket; a second for the flags, the u16 length sum, the offset's low byte and each member's
    (sequence, length) item into its bucket; each bucket sorted by one wave for the visit-order
    samples.  A key whose members crowd one bucket (clustered: each planted key's sequences
    consecutive) takes the round-3 path -- compaction, LSD radix sort of the sequence indices,
    length gathers -- as every key does with heavy_lsd = 1 (Boyer-Moore + recount for the best).
    Planted 8-mers: pure (kept, some sequences hold it three times), exactly 80 % (kept),
    one short of 80 % (cut), a 50/50 tie (cut), and one inside a > 65535-residue protein."""
    rng = np.random.default_rng(44)
    aa = np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY", np.uint8)

    def rnd(k):
        return bytes(rng.choice(aa, k))
    seqs, funcs = [], []
    plan = [(rnd(8), [1] * 5000, True), (rnd(8), [2] * 3200 + [3] * 800, False),
            (rnd(8), [2] * 3199 + [5] * 801, False), (rnd(8), [4] * 2100 + [0] * 2100, False),
            (rnd(8), [0] * 4100, False)]
    for pi, (core, fl, rep) in enumerate(plan):
        rng.shuffle(fl)
        for j, fn in enumerate(fl):
            a, b = rnd(int(rng.integers(0, 400))), rnd(int(rng.integers(0, 400)))
            body = core * 3 if (rep and j % 7 == 0) else core
            if pi == 4 and j == 17:
                a = rnd(70000)
            seqs.append(a + body + b)
            funcs.append(fn)
    order = np.arange(len(seqs)) if clustered else rng.permutation(len(seqs))
    seqs = [seqs[k] for k in order]
    res, off, lens = pack(seqs)
    func = np.array(funcs, np.uint16)[order]
    sid = np.arange(len(seqs), dtype=np.uint32)
    ref = oracle_ref.build(res, off, lens, func, sid, 6)
    b = skm.SignatureBuilder(6)
    if passes:
        b.set_option("key_range_passes", passes)
    b.set_option("giant_class", giant_class)  # 0: off; 11/12: the planted keys' chains start after k_heavy
    b.set_option("heavy_lsd", lsd)
    b.add_batch(res, off, lens, func, sid)
    b.run()
    ovf = b.debug_overflow()
    if giant_class in (11, 12):
        assert b.counters()["giant_chains"] >= 2
    got = b.finish()
    b.close()
    assert_same(got, ref)
    keys = {int.from_bytes(c, "little"): fl for c, fl, _ in plan}
    kept = set(int(k) for k in got.keys)
    assert [k in kept for k in keys] == [True, True, False, False, True]
    if not passes:
        assert max(ovf) >= 4096
