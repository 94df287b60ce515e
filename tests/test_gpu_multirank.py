"""Multi-GPU build semantics on one device: ranks 0..n-1 run in-process (skm_build_group_run,
device-copy exchange in place of the RCCL all-to-all) and must reproduce the single-process
oracle on the union of their shards bit for bit (owner-partitioned exchange)."""
import numpy as np
import pytest

import oracle_ref
from signature_kmers_amd import synth

pytestmark = pytest.mark.gpu


def shard(p, world, rank):
    """rank r gets the r-th contiguous range of files (sequence order = rank order)."""
    files = np.unique(p.file_of)
    mine = np.array_split(files, world)[rank]
    sel = np.isin(p.file_of, mine)
    return sel


def run_group(skm, arrays, nf, world, sel_fn, opts=None, counters=None):
    r, o, l, f, i = arrays
    bs = []
    for rank in range(world):
        sel = sel_fn(rank)
        b = skm.SignatureBuilder(nf, device=0, rank=rank, world_size=world)
        for k, v in (opts or {}).items():
            b.set_option(k, v)
        idx = np.nonzero(sel)[0]
        if len(idx):
            b.add_batch(r, o[idx], l[idx], f[idx], i[idx])
        bs.append(b)
    skm.group_run(bs)
    if counters is not None:
        counters.extend(b.counters() for b in bs)
    outs = [b.finish() for b in bs]
    for b in bs:
        b.close()
    return outs


def check_against_oracle(got, ref):
    np.testing.assert_array_equal(got.keys, ref["keys"])
    np.testing.assert_array_equal(got.data.view(np.uint8), ref["data"].view(np.uint8))
    np.testing.assert_array_equal(got.distinct_functions, ref["distinct_functions"])
    np.testing.assert_array_equal(got.seqs_with_func, ref["seqs_with_func"])
    assert got.n_seqs_with_signature == ref["n_seqs_with_signature"]
    assert got.distinct_signatures == ref["distinct_signatures"]


@pytest.mark.parametrize("world", [2, 4, 8])
def test_group_build_matches_oracle(skm, gpu, world):
    p = synth.generate_arrays(16000, 120, per_file=1000, extras=True)
    r, o, l, f, i, funcs = synth.build_inputs(p)
    ref = oracle_ref.build(r, o, l, f, i, len(funcs))
    outs = run_group(skm, (r, o, l, f, i), len(funcs), world, lambda k: shard(p, world, k))
    check_against_oracle(outs[0], ref)
    # every other rank returns the k-mers it owns; together they partition the kept set
    owned = np.concatenate([x.keys for x in outs[1:]] + [np.zeros(0, np.uint64)])
    assert len(np.intersect1d(owned, outs[0].keys)) == len(owned)
    for x in outs[1:]:
        assert x.distinct_signatures == ref["distinct_signatures"]
        np.testing.assert_array_equal(x.distinct_functions, ref["distinct_functions"])


def test_group_heavy_groups_and_empty_rank(skm, gpu):
    # one heavy k-mer family (deep overflow sub-buckets + long chains) split over ranks, rank 1 empty
    rng = np.random.default_rng(5)
    motif = b"MKVLAAGWQERTY"
    seqs, funcs = [], []
    for k in range(6000):
        pre = bytes(rng.choice(np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY", np.uint8), int(rng.integers(0, 40))))
        seqs.append(pre + motif + pre[::-1])
        funcs.append(int(k % 7 == 0))
    lens = np.array([len(s) for s in seqs], np.uint32)
    off = np.zeros(len(seqs), np.uint64)
    off[1:] = np.cumsum(lens[:-1].astype(np.uint64))
    res = np.frombuffer(b"".join(seqs), np.uint8)
    fn = np.array(funcs, np.uint16)
    ids = np.arange(len(seqs), dtype=np.uint32)
    ref = oracle_ref.build(res, off, lens, fn, ids, 2)
    n = len(seqs)
    bounds = [0, n // 2, n // 2, 3 * n // 4, n]  # rank 1 has no sequences

    def sel(k):
        m = np.zeros(n, bool)
        m[bounds[k]:bounds[k + 1]] = True
        return m

    outs = run_group(skm, (res, off, lens, fn, ids), 2, 4, sel)
    check_against_oracle(outs[0], ref)


def test_group_colliding_seq_ids(skm, gpu):
    p = synth.generate_arrays(3000, 40, per_file=500)
    r, o, l, f, i, funcs = synth.build_inputs(p)
    i = (i % 700).astype(np.uint32)  # ids collide across files and ranks
    ref = oracle_ref.build(r, o, l, f, i, len(funcs))
    outs = run_group(skm, (r, o, l, f, i), len(funcs), 2, lambda k: shard(p, 2, k))
    check_against_oracle(outs[0], ref)


@pytest.mark.parametrize("world,passes,first", [(2, 2, -1), (2, 4, -1), (4, 4, -1), (2, 4, 0), (2, 0, -1)])
def test_group_heavy_key_routing(skm, gpu, world, passes, first):
    """Heavy-key routing at world > 1 (VERDICT r03 missing #1, r04 #4): the ranks' count-min
    sketches are summed and their Bloom filters OR-ed, so every rank routes the same globally heavy
    k-mers.  By default (route_first) they all go to a heavy-only pass 0 -- the light keys of pass 0
    spread over the other passes, every element carrying (natural ^ routed pass) -- so their giant
    chains start a short pass into the step; route_first = 0 keeps round 4's routing into the first
    half.  passes = 0: the pass count from a small memory budget (two passes), doubled to four by
    route_first.  The union is the oracle's bit for bit and every rank routed occurrences."""
    p = synth.generate_arrays(60000, 60, per_file=2000, seed=6)
    r, o, l, f, i, funcs = synth.build_inputs(p)
    ref = oracle_ref.build(r, o, l, f, i, len(funcs))
    ctrs = []
    opts = {"key_range_passes": passes, "route_heavy_min": 256, "main_long_class": 8, "overflow_long_class": 8}
    if first >= 0:
        opts["route_first"] = first
    if first != 0:
        opts["route_first_min"] = 256
    if passes == 0:
        opts["device_memory_budget_mb"] = 1000
    outs = run_group(skm, (r, o, l, f, i), len(funcs), world, lambda k: shard(p, world, k), opts, ctrs)
    check_against_oracle(outs[0], ref)
    for c in ctrs:
        assert c["passes"] == (passes or 4) and c["routed"] > 10_000, c
