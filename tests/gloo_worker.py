"""One rank of a multi-process (torch.distributed gloo) run, launched by tests/test_*gloo*.py via
torch.distributed.run.  Modes:
  plan   host only: skm_debug_transport_check + the exchange planning of skm_build over the gloo
         host transport, checked against numpy on the gathered inputs of every rank;
  build  rank r builds the r-th contiguous file range on cuda:0 (every rank shares the one GPU),
         exchanging through the gloo host transport; rank 0's kept set and statistics must equal
         the oracle on the union (one pass, two key-range passes, and two / four with heavy-key
         routing);
  matrix rank r looks up its range of the queries for kmers-matrix-distance, hits go to their
         k-mer's owner and groups to the row bands they touch over the gloo transport; the bands
         concatenated equal the oracle's pairs.
Writes <out>/ok.<rank> on success."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def plan(skm, dist, rank, world):
    import torch
    T = skm.GlooTransport()
    assert skm.lib().skm_debug_transport_check(T.ptr, rank, world) == 0, skm.lib().skm_last_error()
    for nb1, seed in ((16, 1), (4096, 2)):
        rng = np.random.default_rng([seed, rank])
        counts = rng.integers(0, 50, size=world * nb1).astype(np.uint64)
        counts[rng.random(len(counts)) < 0.2] = 0  # empty buckets and (sometimes) empty peers
        starts = np.zeros(world * nb1 + 1, np.uint64)
        starts[1:] = np.cumsum(counts)
        ro = np.zeros(world, np.uint64)
        rc = np.zeros(world, np.uint64)
        vs = np.zeros(nb1 + 1, np.uint64)
        P = skm._ptr
        rc_ = skm.lib().skm_debug_exchange_plan(T.ptr, rank, world, nb1, P(starts), P(ro), P(rc), P(vs))
        assert rc_ == 0, skm.lib().skm_last_error()
        allc = [torch.zeros(world * nb1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(allc, torch.from_numpy(counts.astype(np.int64)))
        recv = np.stack([c.numpy()[rank * nb1:(rank + 1) * nb1] for c in allc])  # [source][bucket]
        want_cnt = recv.sum(axis=1)
        assert np.array_equal(rc, want_cnt)
        assert np.array_equal(ro, np.concatenate([[0], np.cumsum(want_cnt)[:-1]]))
        assert np.array_equal(vs, np.concatenate([[0], np.cumsum(recv.sum(axis=0))]))


def build(skm, dist, rank, world):
    import oracle_ref
    from signature_kmers_amd import synth
    p = synth.generate_arrays(12000, 80, per_file=1000, extras=True, seed=11)
    r, o, l, f, i, funcs = synth.build_inputs(p)
    files = np.array_split(np.unique(p.file_of), world)[rank]
    idx = np.nonzero(np.isin(p.file_of, files))[0]
    ref = oracle_ref.build(r, o, l, f, i, len(funcs)) if rank == 0 else None
    T = skm.GlooTransport()
    for passes, route, first in ((1, 0, 1), (2, 0, 1), (2, 64, 1), (4, 64, 1), (4, 64, 0)):
        # route > 0: heavy-key routing over the transport (summed sketches, OR-ed filters); first:
        # into a heavy-only pass 0 (the world > 1 default), else into the first half of the passes
        b = skm.SignatureBuilder(len(funcs), device=0, rank=rank, world_size=world)
        b.set_option("key_range_passes", passes)
        b.set_option("route_heavy_min", route)
        b.set_option("route_first_min", route or 1 << 17)
        b.set_option("route_first", first)
        if len(idx):
            b.add_batch(r, o[idx], l[idx], f[idx], i[idx])
        b.set_transport(T)
        b.run()
        got = b.finish()
        c = b.counters()
        b.close()
        assert c["passes"] == passes
        assert (c["routed"] > 0) == (route > 0 and passes > 1), c
        if rank == 0:
            assert np.array_equal(got.keys, ref["keys"])
            assert np.array_equal(got.data.view(np.uint8), ref["data"].view(np.uint8))
            assert np.array_equal(got.distinct_functions, ref["distinct_functions"])
            assert np.array_equal(got.seqs_with_func, ref["seqs_with_func"])
            assert got.n_seqs_with_signature == ref["n_seqs_with_signature"]
            assert got.distinct_signatures == ref["distinct_signatures"]
        else:
            assert got.distinct_signatures == len(ref["keys"]) if ref else True


def matrix(skm, dist, rank, world):
    """Multi-GPU kmers-matrix-distance over the gloo host transport: rank r looks up its contiguous
    range of the queries, hits go to their k-mer's owner, groups to the row bands they touch; the
    bands concatenated in rank order equal the oracle's pairs over all queries (SeqIdMap indices
    global, some shared across the rank boundary)."""
    import oracle_ref
    from signature_kmers_amd import synth
    p = synth.generate_arrays(3000, 30, per_file=500, seed=41)
    r, o, l, f, i, funcs = synth.build_inputs(p)
    ref = oracle_ref.build(r, o, l, f, i, len(funcs))
    out = sys.argv[2]
    base = os.path.join(out, f"kmer_data.{rank}")
    skm.mph_build(ref["keys"], ref["data"], base + ".mph", base + ".dat", seed=7)  # host builder: same bytes
    q = synth.generate_arrays(40 * 500, 30, per_file=500, first_file=20, n_files=20, seed=41, extras=True)
    n = len(q.seq_len)
    idx = np.arange(n, dtype=np.uint32)
    for s in range(7, n, 7):  # SeqIdMap: repeated ids share an index (across rank boundaries too)
        idx[s] = idx[s - 3]
    _, idx = np.unique(idx, return_inverse=True)  # first-appearance order == sorted order here
    idx = idx.astype(np.uint32)
    nidx = int(idx.max()) + 1
    part = np.array_split(np.arange(n), world)[rank]
    a, b = int(part[0]), int(part[-1]) + 1
    db = skm.CmphKmerDb(base, device=0)
    md = skm.MatrixDistance(db, funcs, q.residues, q.seq_off[a:b], q.seq_len[a:b], seq_idx=idx[a:b], n_idx=nidx)
    md.set_transport(skm.GlooTransport())
    got = md.compute()
    c = md.counters()
    lo, hi = skm.matrix_tile_rows(nidx, rank, world)
    assert len(got) == 0 or (got[:, 0].min() >= lo and got[:, 0].max() < hi)
    md.run()  # collective again on the same handle: the same band
    assert np.array_equal(md.pairs(), got)
    md.close()
    db.close()
    parts = [None] * world
    dist.all_gather_object(parts, got)
    ctrs = [None] * world
    dist.all_gather_object(ctrs, c)
    if rank == 0:
        allp = np.concatenate(parts)
        ob = oracle_ref.Bdz(open(base + ".mph", "rb").read())
        exp = oracle_ref.matrix_distance(ob, open(base + ".dat", "rb").read(), q.residues, q.seq_off, q.seq_len, idx,
                                         funcs.index("hypothetical protein"))
        assert len(exp) > 10000
        assert np.array_equal(allp, exp), (len(allp), len(exp))
        assert sum(x["increments"] for x in ctrs) == int(exp[:, 2].astype(np.int64).sum())


def main():
    mode, out = sys.argv[1], sys.argv[2]
    import torch.distributed as dist
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    import signature_kmers_amd as skm
    {"plan": plan, "build": build, "matrix": matrix}[mode](skm, dist, rank, world)
    dist.barrier()
    open(os.path.join(out, f"ok.{rank}"), "w").write("ok\n")
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
