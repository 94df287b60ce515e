#!/usr/bin/env python3
"""bench.py -- signature-k-mer build throughput on MI355X (BASELINE.json metric).

Metric: k-mers/sec (windows examined by extract+hash+count+cut), whole job over N GPUs.
Workload at N=1: BASELINE configs[1] -- 1M synthetic protein sequences, k=8, signature build on
one MI355X (SURVEY.md 8(d) generator, seed 20241115).  At N>1 (weak scaling) rank r holds the
r-th contiguous range of files of an N x 1M proteome and the ranks run ONE build over the union:
occurrence elements go to the owner GPU of their k-mer with an RCCL all-to-all over xGMI, then
per-function counts and signature flags are all-reduced.

One step = one full device pass of the build pipeline over the HBM-resident input
(extract/count, scan, extract/scatter, bucket group-by + cut + statistics, overflow, stats).
Inputs are uploaded before the timed region; outputs stay on the device.

Launch: python bench.py [--gpus N --steps K --warmup W]   (N>1 under torch.distributed.run)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s peak


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--seqs", type=int, default=1_000_000, help="sequences per GPU")
    ap.add_argument("--families", type=int, default=4000)
    ap.add_argument("--cpu-sample-seqs", type=int, default=1_000_000,
                    help="sequences of the workload the CPU baseline builds (default: all of C2)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="host threads of the CPU baseline (0: OMP_NUM_THREADS, else min(16, cores))")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--annot-queries", type=int, default=2_000_000,
                    help="annotate leg (BASELINE configs[3] at reduced query count; 0 = off; N=1 only)")
    ap.add_argument("--matrix-seqs", type=int, default=100_000,
                    help="matrix-distance leg (BASELINE configs[4]: all-vs-all over this many query "
                         "sequences of 200 families; 0 = off; N=1 only)")
    return ap.parse_args()


def main():
    a = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    import signature_kmers_amd as skm
    from signature_kmers_amd import synth
    uid = None
    if world > 1:
        import torch.distributed as dist  # gloo: rendezvous, barrier, max over ranks (host side)
        dist.init_process_group("gloo")
        box = [skm.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        uid = box[0]

    # ---- synthetic shard (one RNG stream per file: shards are rank-independent) ----
    per_file = 4000
    files_per_rank = (a.seqs + per_file - 1) // per_file
    t0 = time.time()
    p = synth.generate_arrays(a.seqs * world, a.families, per_file=per_file, first_file=rank * files_per_rank,
                              n_files=files_per_rank)
    r, o, l, f, i, funcs = synth.build_inputs(p)
    gen_s = time.time() - t0
    n_windows = int(np.where((f != 0xFFFF) & (l >= 8), l.astype(np.int64) - 7, 0).sum())

    ndev = max(1, skm.device_count())
    b = skm.SignatureBuilder(len(funcs), device=local % ndev, rank=rank, world_size=world)
    b.add_batch(r, o, l, f, i)
    if uid is not None:
        b.set_comm(uid)  # RCCL communicator over the world (data-path exchange)
    b.prepare()

    def barrier():
        if dist is not None:
            dist.barrier()

    for _ in range(a.warmup):
        b.run()
    phase = {}
    barrier()
    t1 = time.perf_counter()
    for _ in range(a.steps):
        b.run()
        for k, v in b.timings().items():
            phase[k] = phase.get(k, 0.0) + v
    t_local = time.perf_counter() - t1  # run() returns after its final event has completed
    barrier()
    t_max = t_local
    if dist is not None:
        import torch
        tt = torch.tensor([t_local], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t_max = float(tt.item())
        nw = torch.tensor([n_windows], dtype=torch.float64)
        dist.all_reduce(nw, op=dist.ReduceOp.SUM)
        total_windows = float(nw.item())
    else:
        total_windows = float(n_windows)
    ms_per_step = 1000.0 * t_max / a.steps
    value = total_windows * a.steps / t_max
    phase = {k: v / a.steps for k, v in phase.items()}

    # ---- roofline: dominant kernel (bucket group-by) and the whole pipeline ----
    res_bytes = int(len(r) + len(l))
    valid = _valid_windows(r, o, l, f)          # occurrence elements this rank extracts
    ctrs = b.counters()
    grouped = ctrs["grouped"]                   # elements this rank groups (after the exchange)
    n_kept = ctrs["kept"]                       # kept k-mers this rank owns
    # dominant single kernel: k_bucket_process (group-by + cut + statistics of every sub-bucket
    # that fits LDS).  Its algorithmic bytes: the 16-byte elements it reads once, the 18 bytes per
    # k-mer it keeps; the overflow sub-buckets (k_overflow) and the k-mers of groups of > 64
    # members (kept by k_big_groups) are excluded.
    kernels = {"k_extract<false>": "extract_count", "k_partition": "partition", "k_bucket_process": "bucket_kernel"}
    dom = max(kernels, key=lambda k: phase.get(kernels[k], 0.0))
    alg = {
        "k_extract<false>": res_bytes,
        "k_partition": 32 * grouped,  # 16-byte elements read once and written once
        "k_bucket_process": 16 * (grouped - ctrs["overflow_elements"])
        + 18 * (n_kept - ctrs["overflow_kept"] - ctrs["big_kept"]),
    }
    dom_ms = phase[kernels[dom]]
    achieved = alg[dom] / (dom_ms * 1e-3) / 1e9
    pipe_alg = res_bytes + 16 * valid + 16 * grouped + 18 * n_kept  # SURVEY 8(d) B_alg
    pipe_gbs = pipe_alg / (phase["total"] * 1e-3) / 1e9
    traffic = _pmc_traffic(dom, a.seqs)

    out = {
        "metric": "k-mers/sec (extract+hash+count) at 1/2/4/8 GPUs; achieved HBM GB/s %",
        "value": value,
        "unit": "k-mers/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (SURVEY 8(d) generator, seed 20241115)",
        "config": {"workload": "C2: 1M protein seqs/GPU, k=8, signature build (extract+group+cut+stats)",
                   "seqs_per_gpu": a.seqs, "families": a.families, "windows_per_gpu": n_windows,
                   "valid_windows_per_gpu": valid, "kept_kmers_rank0": n_kept, "grouped_elements_rank0": grouped,
                   "parallelism": "single GPU" if world == 1 else
                   f"{world} GPUs, owner-partitioned RCCL all-to-all + all-reduce"},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "alg_bytes_per_launch": alg[dom], "avg_launch_ms": dom_ms},
        "pipeline": {"alg_bytes": pipe_alg, "ms": phase["total"], "GBs": pipe_gbs, "frac": pipe_gbs / HBM_PEAK_GBS,
                     "phase_ms": phase},
        "cpu_baseline": None,
        "gen_seconds": gen_s,
    }
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = _cpu_baseline(r, o, l, f, i, len(funcs), a.cpu_sample_seqs, a.cpu_threads)
    if world == 1 and a.annot_queries > 0:
        out["annotate"] = _annotate_leg(skm, synth, b, funcs, a, files_per_rank, local % ndev)
    b.close()
    if world == 1 and a.matrix_seqs > 0:
        out["matrix"] = _matrix_leg(skm, synth, a, local % ndev)
    if rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as fh:
                fh.write(line + "\n")
    if dist is not None:
        dist.destroy_process_group()


def _annotate_leg(skm, synth, b, funcs, a, files_train, device):
    """kmers-call-functions path (BASELINE configs[3]): fresh query proteins of the same families
    (files after the training set: their own RNG streams) against the CMPH/BDZ DB of this build,
    resident in HBM.  One step = window lookup (k_lookup) + HitSet calls + compaction over every
    query; the calls stay on the device.  Roofline: k_lookup, SURVEY 8(d) B_alg = 1 B/residue +
    18 B/window (g bytes, rank word, record)."""
    import tempfile
    kept = b.finish()
    t0 = time.time()
    nq = a.annot_queries
    per_file = 4000
    p = synth.generate_arrays(a.seqs + nq, a.families, per_file=per_file, first_file=files_train,
                              n_files=(nq + per_file - 1) // per_file)
    gen_s = time.time() - t0
    with tempfile.TemporaryDirectory(dir="/tmp") as d:
        base = os.path.join(d, "kmer_data")
        t0 = time.time()
        skm.mph_build(kept.keys, kept.data, base + ".mph", base + ".dat", seed=1, device=device)
        mph_s = time.time() - t0
        db = skm.CmphKmerDb(base, device=device)
        files = None if a.no_cpu_baseline else (open(base + ".mph", "rb").read(), open(base + ".dat", "rb").read())
    hypo = funcs.index("hypothetical protein")
    q = skm.QueryBatch(db, p.residues, p.seq_off, p.seq_len)
    nwin = int(np.where(p.seq_len >= 8, p.seq_len.astype(np.int64) - 7, 0).sum())
    for _ in range(max(1, a.warmup)):
        q.run(hypo)
    steps = max(3, a.steps)
    acc = {}
    t1 = time.perf_counter()
    for _ in range(steps):
        q.run(hypo)
        for k, v in q.timings().items():
            acc[k] = acc.get(k, 0.0) + v
    wall = time.perf_counter() - t1
    acc = {k: v / steps for k, v in acc.items()}
    off, calls = q.calls()
    q.close()
    db.close()
    alg = int(len(p.residues)) + 18 * nwin
    gbs = alg / (acc["lookup"] * 1e-3) / 1e9
    cpu = None
    if files is not None:  # the call path of the oracle on the host cores, bounded sample
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_ref
        threads = _cpu_threads(a.cpu_threads)
        n = min(len(p.seq_len), 200_000)
        end = int(p.seq_off[n - 1]) + int(p.seq_len[n - 1])
        ob = oracle_ref.Bdz(files[0])
        t = time.perf_counter()
        oracle_ref.annotate_mt(ob, files[1], p.residues[:end], p.seq_off[:n], p.seq_len[:n], threads, hypo_index=hypo)
        dt = time.perf_counter() - t
        w = int(np.where(p.seq_len[:n] >= 8, p.seq_len[:n].astype(np.int64) - 7, 0).sum())
        cpu = {"value": w / dt, "unit": "k-mers/s", "cores": threads, "kind": "port",
               "sample": f"first {n} query proteins ({w} windows), {dt:.1f} s, oracle/skm_oracle.cpp "
                         f"oracle_annotate_mt (process_aa_seq per sequence) on {threads} host threads"}
        del ob, files
    return {"metric": "query k-mers/sec (window lookup + HitSet calls)", "value": nwin * steps / wall,
            "unit": "k-mers/s", "ms_per_step": 1000.0 * wall / steps,
            "config": {"workload": f"C4 at {nq} queries (configs[3] names 10M): fresh proteins of the same "
                                   f"families vs the CMPH DB of this build in HBM", "queries": nq,
                       "windows": nwin, "db_keys": int(len(kept.keys)), "calls": int(len(calls))},
            "phase_ms": acc,
            "roofline": {"bound": "hbm", "kernel": "k_lookup<0>", "achieved": gbs, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS, "alg_bytes_per_launch": alg,
                         "avg_launch_ms": acc["lookup"], "traffic": _pmc_traffic("k_lookup<0>", a.seqs)},
            "cpu_baseline": cpu, "mph_build_s": mph_s, "query_gen_s": gen_s}


def _matrix_leg(skm, synth, a, device):
    """kmers-matrix-distance (BASELINE configs[4]): a 200-family signature DB (built on this GPU from
    200K training proteins, BDZ on the GPU) resident in HBM, a fresh set of query proteins of the
    same families, all-vs-all shared-signature-k-mer counts (one GPU computes every row).  One step =
    window lookup + length filter, k-mer grouping (hash + radix sort), per-row LDS histograms of the
    pair increments, compaction of the nonzero pairs in row order; the pairs stay on the device.
    Roofline: k_md_rows (the pair increments), SURVEY 8(d) 4 B per pair increment."""
    import tempfile
    fam, per_file, n_train = 200, 4000, 200_000
    t0 = time.time()
    p = synth.generate_arrays(n_train, fam, per_file=per_file)
    r, o, l, f, i, funcs = synth.build_inputs(p)
    b = skm.SignatureBuilder(len(funcs), device=device)
    b.add_batch(r, o, l, f, i)
    kept = b.finish()
    b.close()
    nq = a.matrix_seqs
    f0 = n_train // per_file
    nfq = (nq + per_file - 1) // per_file
    q = synth.generate_arrays((f0 + nfq) * per_file, fam, per_file=per_file, first_file=f0, n_files=nfq)
    n = min(nq, len(q.seq_len))
    end = int(q.seq_off[n - 1]) + int(q.seq_len[n - 1])
    res, off, ln = q.residues[:end], q.seq_off[:n], q.seq_len[:n]
    with tempfile.TemporaryDirectory(dir="/tmp") as d:
        base = os.path.join(d, "kmer_data")
        skm.mph_build(kept.keys, kept.data, base + ".mph", base + ".dat", seed=1, device=device)
        db = skm.CmphKmerDb(base, device=device)
        files = None if a.no_cpu_baseline else (open(base + ".mph", "rb").read(), open(base + ".dat", "rb").read())
    prep_s = time.time() - t0
    md = skm.MatrixDistance(db, funcs, res, off, ln)
    for _ in range(max(1, a.warmup)):
        md.run()
    steps = max(3, a.steps)
    acc = {}
    t1 = time.perf_counter()
    for _ in range(steps):
        md.run()
        for k, v in md.timings().items():
            acc[k] = acc.get(k, 0.0) + v
    wall = time.perf_counter() - t1
    acc = {k: v / steps for k, v in acc.items()}
    c = md.counters()
    md.close()
    db.close()
    alg = 4 * c["increments"]
    gbs = alg / (acc["pairs"] * 1e-3) / 1e9
    cpu = None
    if files is not None:  # the oracle's matrix distance (single thread) on a bounded sample
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_ref
        ns = min(n, 10_000)
        e2 = int(off[ns - 1]) + int(ln[ns - 1])
        ob = oracle_ref.Bdz(files[0])
        t = time.perf_counter()
        oracle_ref.matrix_distance(ob, files[1], res[:e2], off[:ns], ln[:ns], np.arange(ns, dtype=np.uint32),
                                   funcs.index("hypothetical protein"))
        dt = time.perf_counter() - t
        w = int(np.where(ln[:ns] >= 8, ln[:ns].astype(np.int64) - 7, 0).sum())
        cpu = {"value": w / dt, "unit": "k-mers/s", "cores": 1, "kind": "port",
               "sample": f"all-vs-all over the first {ns} query proteins ({w} windows; pair work grows with the "
                         f"square of the sample, so this rate is an upper bound for 100K), {dt:.1f} s, "
                         f"oracle/skm_oracle.cpp oracle_matrix_distance, one thread"}
        del ob, files
    return {"metric": "query k-mers/sec (lookup + all-vs-all shared signature k-mer counts)",
            "value": c["windows"] * steps / wall, "unit": "k-mers/s", "ms_per_step": 1000.0 * wall / steps,
            "pair_increments_per_s": c["increments"] / (acc["pairs"] * 1e-3),
            "config": {"workload": f"C5: {n} query proteins of {fam} families, all-vs-all, 1 GPU (one tile)",
                       "queries": n, "families": fam, "db_keys": int(len(kept.keys)), "windows": c["windows"],
                       "hits": c["hits"], "pair_increments": c["increments"], "nonzero_pairs": c["pairs"]},
            "phase_ms": acc,
            "roofline": {"bound": "hbm", "kernel": "k_md_rows", "achieved": gbs, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS, "alg_bytes_per_launch": alg,
                         "avg_launch_ms": acc["pairs"], "traffic": _pmc_traffic("k_md_rows", a.seqs)},
            "cpu_baseline": cpu, "prep_s": prep_s}


def _valid_windows(r, o, l, f) -> int:
    """Count of windows whose 8 residues are all in ok_prot_ (records the build materialises)."""
    ok = np.zeros(256, bool)
    ok[np.frombuffer(b"ACDEFGHIKLMNPQRSTVWYacdefghiklmnpqrstvwy", np.uint8)] = True
    good = ok[r].astype(np.int32)
    c = np.concatenate([[0], np.cumsum(good)])
    total = 0
    for s0, ln, fn in zip(o.astype(np.int64), l.astype(np.int64), f):
        if fn == 0xFFFF or ln < 8:
            continue
        w = c[s0 + 8:s0 + ln + 1] - c[s0:s0 + ln - 7]
        total += int((w == 8).sum())
    return total


def _pmc_traffic(kernel: str, seqs: int):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (profiles/pmc_traffic.json),
    when it was measured on this kernel and workload; else None."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(path))
        e = d["kernels"][kernel]
        if int(d.get("seqs_per_gpu", -1)) != seqs:
            return None
        return e["hbm_bytes_per_launch"]
    except Exception:
        return None


def _cpu_threads(threads: int) -> int:
    if threads <= 0:
        threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    return threads


def _cpu_baseline(r, o, l, f, i, nf, n_sample, threads):
    """The CPU port of the build (oracle/skm_oracle.cpp oracle_build_mt: the --n-threads 1 results
    computed on all the host cores this job owns -- extract into key-hash shards, per-shard stable
    sort + group + cut + statistics) on the first n_sample sequences of the same workload."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ref
    threads = _cpu_threads(threads)
    n = min(n_sample, len(l))
    end = int(o[n - 1]) + int(l[n - 1])
    t = time.perf_counter()
    oracle_ref.build_mt(r[:end], o[:n], l[:n], f[:n], i[:n], nf, threads, sort=False)
    dt = time.perf_counter() - t
    w = oracle_ref.count_windows(l[:n], f[:n])
    return {"value": w / dt, "unit": "k-mers/s", "cores": threads, "kind": "port",
            "sample": f"first {n} sequences of the same workload ({w} windows), {dt:.1f} s, "
                      f"oracle/skm_oracle.cpp oracle_build_mt on {threads} host threads "
                      f"(--n-threads 1 results; unsorted output like the reference's hash map)"}


if __name__ == "__main__":
    main()
