#!/usr/bin/env python3
"""bench.py -- signature-k-mer build throughput on MI355X (BASELINE.json metric).

Metric: k-mers/sec (windows examined by extract+hash+count+cut), whole job over N GPUs.

Headline workload (north_star / BASELINE configs[2], strong scaling): the 50M-protein synthetic
proteome (SURVEY.md 8(d) generator, seed 20241115, 4,000 families, 12,500 genome files of 4,000
proteins) built on N GPUs of one node.  Rank r holds the r-th contiguous range of files; the
ranks run ONE build over the union: each key-range pass extracts the rank's occurrences of that
pass's k-mer range, sends them to the k-mer's owner GPU (RCCL all-to-all over xGMI), groups
and cuts them there; per-function counts and signature flags are all-reduced at the end
(SURVEY.md 8(e)).  On one GPU the 16.2 G occurrences exceed HBM, so the build runs as key-range
passes over the resident residues (include/skm.h skm_build_set_option "key_range_passes").

One step = one full device pass of the build over the HBM-resident input (pass ids, per pass:
extract/count, scan, extract/scatter, [exchange], partition, group-by + cut + statistics,
overflow, chains; then statistics and reductions).  Inputs are uploaded before the timed region;
outputs stay on the device.

Secondary lines (same JSON object): "weak" = C2 (1M proteins per GPU; configs[1] at N=1) with its
own roofline; at N=1 also the annotate leg (configs[3]: 10M queries vs the C2 DB in HBM) and the
matrix-distance leg (configs[4]).

Launch: python bench.py [--gpus N --steps K --warmup W]   (N>1 under torch.distributed.run)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

# libskm drives up to 12 streams per build (two overflow streams, stashed, per-lane and giant chain
# streams);
# HIP maps streams onto GPU_MAX_HW_QUEUES hardware queues (default 4), read at HIP init
# (SKM_HW_QUEUES: an explicit count for A/B runs)
if os.environ.get("SKM_HW_QUEUES"):
    os.environ["GPU_MAX_HW_QUEUES"] = os.environ["SKM_HW_QUEUES"]
elif int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < 16:
    os.environ["GPU_MAX_HW_QUEUES"] = "16"

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s peak
PER_FILE = 4000
C2_SEQS = 1_000_000


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--seqs-total", type=int, default=50_000_000,
                    help="proteins of the headline proteome, split over the GPUs (strong scaling)")
    ap.add_argument("--families", type=int, default=4000)
    ap.add_argument("--weak-seqs", type=int, default=C2_SEQS,
                    help="proteins per GPU of the secondary weak-scaling (C2) line; 0 = off")
    ap.add_argument("--cpu-shard-div", type=int, default=8,
                    help="the C3 CPU baseline builds the first 1/N shard of the proteome (SURVEY 8(d): 1/8)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="host threads of the CPU baseline (0: all usable)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--gen-workers", type=int, default=0, help="generator processes (0: usable cores)")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--cache-dir", default=None, help="save / reuse the generated headline shard (profiling)")
    ap.add_argument("--cache-only", action="store_true", help="generate + cache every input of this run (headline shard, queries, matrix sets), then exit")
    ap.add_argument("--option", action="append", default=[],
                    help="name=value: skm_build_set_option on the headline build (experiments)")
    ap.add_argument("--annot-queries", type=int, default=10_000_000,
                    help="annotate leg (BASELINE configs[3]); 0 = off; N=1 only")
    ap.add_argument("--recall", type=int, default=1,
                    help="recall leg (SURVEY 8(f)2: the C2 training set vs its exact kept-k-mer DB); 0 = off; N=1 only")
    ap.add_argument("--matrix-seqs", type=int, default=100_000,
                    help="matrix-distance leg (BASELINE configs[4]); 0 = off; owner-partitioned over the ranks")
    ap.add_argument("--cli-seqs", type=int, default=1_000_000,
                    help="cli_build leg: bin/kmers-build-signatures end to end on FASTA directories of this many "
                         "proteins (BASELINE configs[1]); 0 = off; N=1 only")
    ap.add_argument("--cli-queries", type=int, default=10_000_000,
                    help="cli_call leg: bin/kmers-call-functions end to end on this many query proteins (FASTA) "
                         "against the cli_build leg's DB (BASELINE configs[3]); 0 = off")
    ap.add_argument("--mph", type=int, default=1,
                    help="with --finish: the device BDZ over the whole headline kept set, checked on the device; N=1")
    ap.add_argument("--finish", type=int, default=1,
                    help="time skm_build_finish (the kept-set hand-off to host arrays) on the headline build; N=1")
    ap.add_argument("--comm", choices=("rccl", "host"), default="rccl",
                    help="rank exchange of the build: RCCL over xGMI, or the gloo host transport (rehearses the "
                         "multi-rank path with several ranks on one GPU)")
    return ap.parse_args()


def host_cores() -> dict:
    """CPUs this process may use: the affinity mask, capped by a cgroup CPU quota when one is
    set (the GPU boxes give each job a 16-CPU quota on a larger machine), plus the CPU model."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = int(q) // int(p)
    except (OSError, ValueError):
        pass
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    usable = min(aff, quota) if quota else aff
    return {"usable": max(1, usable), "affinity": aff, "cgroup_quota": quota, "model": model}


_T0 = time.time()


def log(msg: str):
    """Progress on stderr (the GPU harness takes a silent run for a hung one)."""
    print(f"[bench {time.time() - _T0:7.1f}s] {msg}", file=sys.stderr, flush=True)


def _windows(lens) -> int:
    return int(np.where(lens >= 8, lens.astype(np.int64) - 7, 0).sum())


class Shard:
    """Per-file generator output of one rank (SURVEY 8(d) arrays, file order)."""

    def __init__(self, parts):
        self.parts = parts
        self.n_seqs = sum(len(p[2]) for p in parts)
        self.n_windows = sum(_windows(p[2]) for p in parts)
        self.n_residues = sum(len(p[0]) for p in parts)

    def add_to(self, b):
        b.reserve(self.n_residues, self.n_seqs)  # one HBM residue buffer; batches stream into it
        for r, o, l, f, i in self.parts:
            b.add_batch(r, o, l, f, i)

    def packed(self, first_files=None):
        ps = self.parts if first_files is None else self.parts[:first_files]
        r = np.concatenate([p[0] for p in ps])
        lens = np.concatenate([p[2] for p in ps])
        off = np.zeros(len(lens), np.uint64)
        if len(lens):
            off[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        return (r, off, lens, np.concatenate([p[3] for p in ps]), np.concatenate([p[4] for p in ps]))


def gen(synth, n_total, families, first_file, n_files, workers, cache=None):
    """The rank's files; with cache (a directory) they are saved on first use and memory-mapped
    afterwards (profiling runs: generator pools do not run under rocprofv3)."""
    tag = f"{n_total}_{families}_{first_file}_{n_files}"
    if cache and os.path.exists(os.path.join(cache, tag + ".res.npy")):
        res = np.load(os.path.join(cache, tag + ".res.npy"), mmap_mode="r")
        meta = np.load(os.path.join(cache, tag + ".meta.npz"))
        lens, func, ids, nper = meta["lens"], meta["func"], meta["ids"], meta["nper"]
        parts, so, ro = [], 0, 0
        for n in nper:
            ln = lens[so:so + n]
            off = np.zeros(n, np.uint64)
            if n:
                off[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
            tot = int(ln.sum())
            parts.append((res[ro:ro + tot], off, ln, func[so:so + n], ids[so:so + n]))
            so += n
            ro += tot
        return Shard(parts)
    sh = Shard(list(synth.iter_file_inputs(n_total, families, PER_FILE, first_file, n_files, workers=workers)))
    if cache:
        os.makedirs(cache, exist_ok=True)
        np.save(os.path.join(cache, tag + ".res.npy"), np.concatenate([p[0] for p in sh.parts]))
        np.savez(os.path.join(cache, tag + ".meta.npz"), lens=np.concatenate([p[2] for p in sh.parts]),
                 func=np.concatenate([p[3] for p in sh.parts]), ids=np.concatenate([p[4] for p in sh.parts]),
                 nper=np.array([len(p[2]) for p in sh.parts], np.int64))
    return sh


def main():
    a = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    cores = host_cores()
    workers = a.gen_workers or min(16, cores["usable"])
    if world > 1:
        import torch.distributed as dist  # gloo: rendezvous, barrier, max over ranks (host side)
        dist.init_process_group("gloo")
        workers = max(1, workers // min(world, 8))
    from signature_kmers_amd import synth

    # ---- every input this rank needs, generated BEFORE any GPU call (the pool spawns processes) ----
    t0 = time.time()
    files_total = (a.seqs_total + PER_FILE - 1) // PER_FILE
    f0, f1 = rank * files_total // world, (rank + 1) * files_total // world
    log(f"rank {rank}/{world}: generating files [{f0}, {f1}) with {workers} workers")
    c3 = gen(synth, a.seqs_total, a.families, f0, f1 - f0, workers, a.cache_dir)
    log(f"generated {c3.n_seqs:,} proteins, {c3.n_windows:,} windows")
    c2_files = (a.weak_seqs + PER_FILE - 1) // PER_FILE
    if a.weak_seqs and f0 == rank * c2_files and f1 - f0 >= c2_files:
        c2 = Shard(c3.parts[:c2_files])  # files [r*250, r*250+250): the same bytes as the weak shard
    elif a.weak_seqs:
        c2 = gen(synth, a.weak_seqs * world, a.families, rank * c2_files, c2_files, workers)
    else:
        c2 = None
    queries = None
    if world == 1 and a.annot_queries > 0:
        nqf = (a.annot_queries + PER_FILE - 1) // PER_FILE
        if c2_files + nqf <= len(c3.parts):  # files after the training set: fresh proteins, own RNG streams
            queries = Shard(c3.parts[c2_files:c2_files + nqf])
        else:
            queries = gen(synth, (c2_files + nqf) * PER_FILE, a.families, c2_files, nqf, workers, a.cache_dir)
    matrix_in = None
    if a.matrix_seqs > 0:  # every rank: the DB is replicated, the pair triangle tiled by rows
        fam, n_train = 200, 200_000
        nfq = (a.matrix_seqs + PER_FILE - 1) // PER_FILE
        tf = n_train // PER_FILE
        matrix_in = (gen(synth, n_train, fam, 0, tf, workers, a.cache_dir),
                     gen(synth, (tf + nfq) * PER_FILE, fam, tf, nfq, workers, a.cache_dir), synth.functions(fam))
    cli_dir = None
    if world == 1 and a.cli_seqs > 0 and not a.cache_only:  # FASTA directories for the CLI legs (spawned writers)
        import tempfile
        cli_dir = tempfile.mkdtemp(prefix="skm_cli_", dir="/tmp")
        t = time.time()
        synth.write_dirs_parallel(os.path.join(cli_dir, "in"), a.cli_seqs, a.families, per_file=PER_FILE,
                                  workers=workers)
        log(f"cli_build input: {a.cli_seqs:,} proteins as FASTA in {time.time() - t:.1f} s")
        if a.cli_queries > 0:  # the query genome files after the training set (the annotate leg's proteins)
            t = time.time()
            qf0 = (a.cli_seqs + PER_FILE - 1) // PER_FILE
            nqf = (a.cli_queries + PER_FILE - 1) // PER_FILE
            synth.write_dirs_parallel(os.path.join(cli_dir, "q"), (qf0 + nqf) * PER_FILE, a.families, per_file=PER_FILE,
                                      workers=workers, first_file=qf0, n_files=nqf)
            log(f"cli_call input: {a.cli_queries:,} query proteins as FASTA in {time.time() - t:.1f} s")
    if a.cache_only:
        log("inputs cached")
        return
    funcs = synth.functions(a.families)
    gen_s = time.time() - t0

    import signature_kmers_amd as skm
    ndev = max(1, skm.device_count())
    device = local % ndev

    def new_uid():
        if world == 1 or a.comm == "host":
            return None
        box = [skm.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        return box[0]

    # ---- headline: C3 strong scaling ----
    uid = new_uid()
    skm.warm_device(device)  # the process's HIP runtime up before the one-shot clock starts
    t0 = time.time()
    b = skm.SignatureBuilder(len(funcs), device=device, rank=rank, world_size=world)
    create_s = time.time() - t0
    for kv in a.option:
        k, v = kv.split("=", 1)
        b.set_option(k, int(v))
    c3.add_to(b)
    if uid is not None:
        b.set_comm(uid)
    elif world > 1:
        b.set_transport(skm.GlooTransport())
    b.prepare()
    prep_s = time.time() - t0
    log(f"C3 prepared in {prep_s:.1f} s")
    head = _measure(skm, b, a.steps, a.warmup, c3, world, dist)
    finish = None
    if world == 1 and a.finish:  # the kept-set hand-off of the headline build (skm_build_finish)
        t = time.perf_counter()
        k = b.finish()
        dt = time.perf_counter() - t
        c = b.counters()
        ok = len(k.keys) == c["kept"] and bool(np.all(k.keys[1:] > k.keys[:-1]))
        finish = {"seconds": dt, "kept": int(len(k.keys)), "bytes": 18 * int(len(k.keys)), "GBs": 18 * len(k.keys) / dt / 1e9,
                  "sorted_and_complete": ok, "chunks": c["finish_chunks"], "host_wait_s": c["finish_wait_us"] / 1e6,
                  "host_copy_s": c["finish_copy_us"] / 1e6,
                  "note": "skm_build_finish: device radix sort in key-range chunks, D2H through pinned staging, "
                          "copied out by the host pool; keys ascending in malloc'd host arrays"}
        log(f"finish (hand-off of {finish['kept']:,} kept k-mers): {dt:.2f} s")
        b.close()
        if a.mph:  # the drop-in build's MPH + .dat over the whole kept set (kmers-build-signatures.cc:253-264)
            t = time.perf_counter()
            st = skm.mph_build_device(k.keys, k.data, None, None, seed=1, device=device, verify=True)
            mph = {"seconds": time.perf_counter() - t, **st,
                   "note": "skm_mph_build_device_ex over the whole headline kept set from host arrays (H2D of keys "
                           "and records included, image files not written): GPU peeling, assignment, rank table, "
                           "record placement, then the on-device check (slots a permutation of [0, n_keys), the "
                           "annotate kernels' pair-line search == bdz_search for every key, .dat[slot] == record)"}
            log(f"mph over {st['n_keys']:,} keys ({st['n_vertices']:,} vertices): {mph['seconds']:.2f} s, "
                f"verified={st['verified']}")
            finish["mph"] = mph
        del k
    b.close()
    per_gpu = a.seqs_total // world
    out = {
        "metric": "k-mers/sec (extract+hash+count) at 1/2/4/8 GPUs; achieved HBM GB/s %",
        "value": head["value"],
        "unit": "k-mers/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": head["ms_per_step"],
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (SURVEY 8(d) generator, seed 20241115)",
        "config": {"workload": f"C3: {a.seqs_total:,}-protein proteome, k=8, signature build "
                               f"(extract+group+cut+stats), {world} GPU(s), ~{per_gpu:,} proteins per GPU",
                   "seqs_total": a.seqs_total, "families": a.families, "windows_total": head["windows_total"],
                   "windows_rank0": c3.n_windows, "key_range_passes": head["passes"],
                   "kept_kmers_rank0": head["counters"]["kept"], "grouped_elements_rank0": head["counters"]["grouped"],
                   "parallelism": "single GPU, key-range passes" if world == 1 else
                   f"{world} GPUs, owner-partitioned {'RCCL' if a.comm == 'rccl' else 'gloo host-transport'} "
                   f"all-to-all + all-reduce, per key-range pass"},
        "roofline": head["roofline"],
        "pipeline": head["pipeline"],
        "value_with_plan": _with_plan(head),
        "pcie_inclusive": _pcie_inclusive(head, prep_s, create_s),
        "finish": finish,
        "cpu_baseline": None,
        "gen_seconds": gen_s,
        "prepare_seconds": prep_s,
    }
    out["chain_tail_ms"] = head["chain_tail_ms"]
    out["giant_chains"] = head["giant_chains"]
    keep = ("overflow_subbuckets", "overflow_elements", "overflow_kept", "big_groups", "big_kept", "chain_jobs",
            "chain_samples", "long_samples", "routed", "pass_groups", "kept_cap", "free_after_prepare", "recs_rot")
    out["build_counters_rank0"] = {k: int(v) for k, v in head["counters"].items() if k in keep}
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        n = a.seqs_total // max(1, a.cpu_shard_div)
        log(f"CPU baseline: first {n:,} proteins (1/{a.cpu_shard_div} shard of C3)")
        out["cpu_baseline"] = _cpu_baseline(
            c3, len(funcs), n, a.cpu_threads or cores["usable"], cores,
            f"the first {n:,} of the {a.seqs_total:,} proteins = one 1/{a.cpu_shard_div} shard "
            f"(genome files 0..{(n + PER_FILE - 1) // PER_FILE - 1}) of the C3 proteome; value is that shard's "
            f"build rate, taken as the extrapolated C3 rate (EXTRAPOLATION, SURVEY 8(d): a shard's k-mer groups are "
            f"~1/{a.cpu_shard_div} the size of the whole proteome's, and the full 15 G-occurrence build does not fit "
            f"the reference's host-memory design)")

    # ---- secondary: C2 per GPU (weak scaling; configs[1] at N=1) ----
    kept = None
    if c2 is not None:
        uid = new_uid()
        b = skm.SignatureBuilder(len(funcs), device=device, rank=rank, world_size=world)
        t0 = time.time()
        c2.add_to(b)
        if uid is not None:
            b.set_comm(uid)
        elif world > 1:
            b.set_transport(skm.GlooTransport())
        b.prepare()
        prep2 = time.time() - t0
        weak = _measure(skm, b, a.steps, a.warmup, c2, world, dist)
        out["weak"] = {"value": weak["value"], "unit": "k-mers/s", "ms_per_step": weak["ms_per_step"],
                       "scaling": "weak",
                       "config": {"workload": f"C2: {a.weak_seqs:,} proteins per GPU x {world}, k=8, signature build",
                                  "windows_total": weak["windows_total"], "kept_kmers_rank0": weak["counters"]["kept"],
                                  "key_range_passes": weak["passes"]},
                       "roofline": weak["roofline"], "pipeline": weak["pipeline"], "chain_tail_ms": weak["chain_tail_ms"],
                       "pcie_inclusive": _pcie_inclusive(weak, prep2), "cpu_baseline": None}
        if rank == 0 and world == 1 and not a.no_cpu_baseline:
            out["weak"]["cpu_baseline"] = _cpu_baseline(
                c2, len(funcs), a.weak_seqs, a.cpu_threads or cores["usable"], cores,
                f"the whole C2 workload ({a.weak_seqs:,} proteins, measured, not extrapolated)")
        if world == 1 and (queries is not None or a.recall):
            kept = b.finish()
        b.close()
    if world == 1 and a.recall and kept is not None and c2 is not None:
        log("recall leg")
        out["recall"] = _recall_leg(skm, kept, funcs, c2, a, device, cores)
    if world == 1 and queries is not None and kept is not None:
        log("annotate leg")
        out["annotate"] = _annotate_leg(skm, kept, funcs, queries, a, device, cores)
    if cli_dir is not None:
        log("cli_build leg")
        out["cli_build"] = _cli_build_leg(cli_dir, a)
        if a.cli_queries > 0 and out["cli_build"].get("rc") == 0:
            log("cli_call leg")
            out["cli_call"] = _cli_call_leg(cli_dir, a)
        import shutil
        shutil.rmtree(cli_dir, ignore_errors=True)
    if matrix_in is not None:
        log("matrix leg")
        mx = _matrix_leg(skm, matrix_in, a, device, cores, rank, world, dist)
        if rank == 0:
            out["matrix"] = mx
    if rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as fh:
                fh.write(line + "\n")
    if dist is not None:
        dist.destroy_process_group()


_ROOF_NOTES = {
    "k_chains_stash": "background stream: the stashed long P^2 / variance chains, one lane each -- serial "
                      "FP64 recurrences in the reference's reverse visit order (SURVEY A.4), so each launch "
                      "lasts as long as its longest chain (~10^6 samples at ~0.6 us) at a few waves per CU; "
                      "latency-bound, not byte-bound: the roofline kernel (the group-by) is the step's byte-moving critical path",
    "k_chains": "P^2 / variance chains (serial FP64 recurrences, one lane each): latency-bound",
    "k_chain_long": "P^2 / variance chains on wave pairs (serial FP64 recurrences): latency-bound",
}


def _alg_bytes(kernel, c, res_bytes):
    """SURVEY 8(d) algorithmic bytes of one build kernel over one step (all its launches), from the
    run's counters; None for a kernel without a stated figure.  c = b.counters()."""
    valid, grouped = c["valid"], c["grouped"]
    table = {
        # the group-by: the 16-byte elements it groups + 18 B per k-mer it keeps (the overflow
        # sub-buckets and the > 64-member groups are other kernels')
        "k_bucket_process": 16 * (grouped - c["overflow_elements"])
        + 18 * (c["kept"] - c["overflow_kept"] - c["big_kept"]),
        "k_partition": 32 * grouped,                       # read + write of each element
        "k_split_stage": 32 * valid,
        "k_extract_stage_pos": res_bytes + 16 * valid,     # residues once + the element written
        "k_extract_stage": res_bytes + 16 * valid,
        "k_extract": res_bytes,
        # per group of passes: the residues once + the group's window positions written
        "k_pass_emit": res_bytes * max(1, c.get("pass_groups", 1)) + 8 * valid,
        "k_pass_hist": 8 * valid,                          # each pass's entries read once
        "k_pass_ids": res_bytes,                           # the per-workgroup pass tally: residues read
        "k_overflow": 16 * c["overflow_elements"],
        "k_ovf_split": 32 * c["overflow_elements"],
        "k_heavy": 16 * c["overflow_elements"],
        # the builder's figure (SURVEY 8(d) states none for the chains): one u32 sample read per
        # recurrence step.  The stashed long chains (key-range passes) run as k_chains_stash (one
        # lane each) or k_chain_long (a wave pair each; the tail batch's longest)
        "k_chain_long": 4 * c["long_samples"],
        "k_chains_stash": 4 * c["long_samples"],
        "k_chains": 4 * (c["chain_samples"] - (c["long_samples"] if c["passes"] > 1 else 0)),
        "k_kept_finalize": 36 * c["kept"],                 # 18 B per kept k-mer read + written
    }
    v = table.get(kernel)
    return None if v is None or v <= 0 else float(v)


def _measure(skm, b, steps, warmup, shard, world, dist):
    """Warmup, then one untimed diagnostic run with every kernel launch bracketed by events (the
    per-kernel GPU time that picks the dominant kernel), then exactly `steps` timed runs bracketed
    by barriers, events around the dominant kernel's launches only; max over ranks."""
    def barrier():
        if dist is not None:
            dist.barrier()

    for w in range(warmup):
        b.run()
        log(f"warmup {w + 1}/{warmup}")
    b.set_kernel_timing(True)
    b.run()
    ktab = b.kernel_timings()
    # the roofline's kernel: the group-by (k_bucket_process), the dominant byte-moving kernel of the
    # main stream that carries the step's critical path; the kernel with the largest GPU time (the
    # background long-chain batches: latency-bound FP64 recurrences at a few waves per CU) is
    # reported beside it (roofline.largest_gpu_time)
    big = max(ktab, key=lambda k: ktab[k][0]) if ktab else None
    dom = "k_bucket_process"
    b.set_kernel_timing(True, dom)
    log(f"roofline kernel: {dom} ({ktab.get(dom, (0, 0))[0]:.1f} ms in {ktab.get(dom, (0, 0))[1]} launches); "
        f"largest GPU time: {big}")
    phase = {}
    dom_ms, dom_n = 0.0, 0
    barrier()
    t1 = time.perf_counter()
    for _ in range(steps):
        b.run()  # returns after the run's final event has completed (device synchronised)
        for k, v in b.timings().items():
            phase[k] = phase.get(k, 0.0) + v
        kt = b.kernel_timings().get(dom, (0.0, 0))
        dom_ms += kt[0]
        dom_n += kt[1]
        log(f"step done ({b.timings()['total']:.1f} ms device)")
    t_local = time.perf_counter() - t1
    barrier()
    b.set_kernel_timing(False)
    ctrs = b.counters()
    t_max, windows_total = t_local, float(shard.n_windows)
    sums = {"grouped": ctrs["grouped"], "kept": ctrs["kept"], "res": shard.n_residues + shard.n_seqs}
    if dist is not None:
        import torch
        tt = torch.tensor([t_local], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t_max = float(tt.item())
        v = torch.tensor([float(shard.n_windows), float(sums["grouped"]), float(sums["kept"]), float(sums["res"])],
                         dtype=torch.float64)
        dist.all_reduce(v, op=dist.ReduceOp.SUM)
        windows_total = float(v[0])
        sums = {"grouped": int(v[1]), "kept": int(v[2]), "res": int(v[3])}
    phase = {k: v / steps for k, v in phase.items()}
    # the dominant kernel (largest GPU time per step over every kernel of the run, measured by the
    # diagnostic run's events): its algorithmic bytes over its launch time in the timed steps
    dom_ms_step = dom_ms / steps
    launches = max(1, dom_n // steps)
    alg = _alg_bytes(dom, ctrs, shard.n_residues + shard.n_seqs)
    achieved = alg / (dom_ms_step * 1e-3) / 1e9 if alg and dom_ms_step > 0 else None
    wl = {50_000_000: "c3", 1_000_000: "c2"}.get(shard.n_seqs, "") if world == 1 else ""
    traffic = _pmc_traffic(dom, wl, shard.n_seqs)
    # SURVEY 8(d) B_alg over the whole job: 1 B/residue + 32 B/valid window + 18 B/kept k-mer
    pipe_alg = sums["res"] + 32 * sums["grouped"] + 18 * sums["kept"]
    pipe_gbs = pipe_alg / (t_max / steps) / 1e9
    top = sorted(ktab.items(), key=lambda kv: -kv[1][0])[:14]
    largest = None
    if big is not None:
        g_ms, g_n = ktab[big]
        g_alg = _alg_bytes(big, ctrs, shard.n_residues + shard.n_seqs)
        g_ach = g_alg / (g_ms * 1e-3) / 1e9 if g_alg and g_ms > 0 else None
        largest = {"kernel": big, "achieved": g_ach, "frac": g_ach / HBM_PEAK_GBS if g_ach else None,
                   "alg_bytes_per_launch": None if g_alg is None else g_alg / max(1, g_n),
                   "avg_launch_ms": g_ms / max(1, g_n), "launches_per_step": g_n,
                   "traffic": (lambda t: None if t is None else t / max(1, g_n))(_pmc_traffic(big, wl, shard.n_seqs)),
                   "note": _ROOF_NOTES.get(big),
                   "timing": "events around each launch in the untimed diagnostic run"}
    return {
        "value": windows_total * steps / t_max,
        "ms_per_step": 1000.0 * t_max / steps,
        "windows_total": int(windows_total),
        "passes": b.passes(),
        "counters": ctrs,
        "roofline": {"bound": "hbm", "kernel": dom, "role": "critical-path kernel (the main stream's group-by)",
                     "largest_gpu_time_kernel": big,
                     "largest_gpu_time_frac": None if largest is None else largest["frac"],
                     "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS if achieved is not None else None,
                     "traffic": None if traffic is None else traffic / launches,
                     "traffic_source": None if traffic is None else f"profiles/{_PMC_FILE} (same libskm sources)",
                     "alg_bytes_per_launch": None if alg is None else alg / launches,
                     "avg_launch_ms": dom_ms_step / launches,
                     "alg_bytes_per_step": alg, "kernel_ms_per_step": dom_ms_step,
                     "launches_per_step": launches,
                     "selection": "the main stream's group-by (the byte-moving kernel on the step's critical "
                                  "path); timed: events around this kernel's launches in the timed steps",
                     "kernels_ms_per_step": {k: round(v[0], 2) for k, v in top},
                     "largest_gpu_time": largest},
        "chain_tail_ms": phase.get("chain_tail"),
        # the run's first giant-chain launch (k_heavy's chains of >= 2^giant_class samples; with
        # route_first the heavy-only pass 0's): start / end from the step's start, rank 0
        "giant_chains": None if phase.get("giant_start", -1) < 0 else {
            "start_ms": phase["giant_start"], "end_ms": phase["giant_end"],
            "chains": ctrs.get("giant_chains"), "longest_samples": ctrs.get("giant_max"),
            "routed_occurrences": ctrs.get("routed")},
        "pipeline": {"alg_bytes": pipe_alg, "ms": 1000.0 * t_max / steps, "GBs": pipe_gbs,
                     "frac": pipe_gbs / HBM_PEAK_GBS / max(1, world), "phase_ms_rank0": phase},
    }


def _with_plan(m):
    """The headline rate with prepare's device pass plan (route sketch, Bloom pack, pass tallies:
    work every build pays once per input) added to the step: reported beside `value`, whose timed
    step reuses the plan."""
    plan = m["counters"].get("prepare_plan_us", 0) / 1e6
    t = m["ms_per_step"] / 1000.0 + plan
    return {"value": m["windows_total"] / t, "unit": "k-mers/s", "plan_s": plan, "step_s": m["ms_per_step"] / 1000.0}


def _cli_build_leg(cli_dir, a):
    """bin/kmers-build-signatures end to end (kmers-build-signatures.cc:126-373) on FASTA directories of
    a.cli_seqs proteins (BASELINE configs[1] at the default): parse + FunctionMap, sequence selection
    and add_batch, prepare, the device build, the kept-set hand-off, final.kmers, the BDZ perfect
    hash + .dat and the recall pass with its reports -- every output file written.  Phases from the
    CLI's own "phases:" stderr line; value = windows built / wall time of the whole process."""
    import shutil
    import subprocess
    exe = os.path.join(ROOT, "bin", "kmers-build-signatures")
    d = os.path.join(cli_dir, "in")
    outd = os.path.join(cli_dir, "kd")
    cmd = [exe, "-D", os.path.join(d, "Annotations"), "-F", os.path.join(d, "Seqs"), "--kmer-data-dir", outd,
           "--final-kmers", "final.kmers", "--perfect-hash", "kmer_data.mph", "--perfect-hash-data", "kmer_data.dat"]
    t = time.perf_counter()
    p = subprocess.run(cmd, capture_output=True, timeout=600)
    wall = time.perf_counter() - t
    res = {"metric": "kmers-build-signatures wall time, FASTA directories -> every output file", "seconds": wall,
           "rc": p.returncode, "config": {"workload": f"C2 CLI: {a.cli_seqs:,} proteins in "
                                                      f"{(a.cli_seqs + PER_FILE - 1) // PER_FILE} FASTA files, 1 GPU"}}
    err = p.stderr.decode(errors="replace")
    if p.returncode != 0:
        res["stderr_tail"] = err[-2000:]
        return res
    ph = [ln for ln in err.splitlines() if ln.startswith("phases: ")]
    if ph:
        f = ph[0].split()[1:]
        res["phases_s"] = {f[i]: float(f[i + 1]) for i in range(0, len(f) - 1, 2)}
    out = p.stdout.decode()
    kept = [ln for ln in out.splitlines() if ln.startswith("Kept ")]
    res["kept"] = int(kept[0].split()[1]) if kept else None
    res["output_bytes"] = {f: os.path.getsize(os.path.join(outd, f)) for f in ("final.kmers", "kmer_data.mph",
                                                                                "kmer_data.dat", "function.index")
                           if os.path.exists(os.path.join(outd, f))}
    shutil.rmtree(os.path.join(cli_dir, "in"), ignore_errors=True)
    return res


def _cli_call_leg(cli_dir, a):
    """bin/kmers-call-functions end to end (kmers-call-functions.cc:84-196) over a.cli_queries query
    proteins in FASTA files against the cli_build leg's kmer_data.mph / .dat (BASELINE configs[3]
    at the default 10M): parse, the device lookup + HitSet calls (skm_annotate, incl. packing,
    upload and the calls' download), host find_best_call on the host pool, the calls file written.
    Phases from the CLI's "phases:" stderr line."""
    import glob
    import subprocess
    exe = os.path.join(ROOT, "bin", "kmers-call-functions")
    files = sorted(glob.glob(os.path.join(cli_dir, "q", "Seqs", "*")))
    outf = os.path.join(cli_dir, "calls.txt")
    cmd = [exe, os.path.join(cli_dir, "kd")] + files + ["-o", outf]
    t = time.perf_counter()
    p = subprocess.run(cmd, capture_output=True, timeout=900)
    wall = time.perf_counter() - t
    res = {"metric": "kmers-call-functions wall time, FASTA files -> calls file", "seconds": wall,
           "rc": p.returncode, "config": {"workload": f"C4 CLI: {a.cli_queries:,} query proteins in {len(files)} "
                                                      f"FASTA files vs the C2 CLI's DB, 1 GPU"}}
    err = p.stderr.decode(errors="replace")
    if p.returncode != 0:
        res["stderr_tail"] = err[-2000:]
        return res
    ph = [ln for ln in err.splitlines() if ln.startswith("phases: ")]
    if ph:
        f = ph[0].split()[1:]
        res["phases_s"] = {f[i]: float(f[i + 1]) for i in range(0, len(f) - 1, 2)}
    res["calls_bytes"] = os.path.getsize(outf) if os.path.exists(outf) else None
    return res


def _pcie_inclusive(m, prep_s, create_s=None):
    """The rate from host arrays: add_batch (packing into the pinned double-buffered staging whose
    DMA to HBM overlaps the packing) + prepare + one build step.  Reported beside `value`, which
    starts with the inputs resident in HBM.  `phases` splits the host time: the handle's creation
    (streams, pinned staging; the process's HIP runtime is initialised before), add_batch (of it:
    packing on the host pool, waiting for a staging buffer's DMA), and
    prepare's residue / metadata upload, pass plan (device tallies + routing sketch) and the rest."""
    t = prep_s + m["ms_per_step"] / 1000.0
    c = m["counters"]
    phases = {"create_s": create_s, "add_batch_s": c.get("add_batch_us", 0) / 1e6,
              "add_pack_s": c.get("add_pack_us", 0) / 1e6, "add_dma_wait_s": c.get("add_dma_wait_us", 0) / 1e6,
              "prepare_upload_s": c.get("prepare_upload_us", 0) / 1e6,
              "prepare_plan_device_s": c.get("prepare_plan_us", 0) / 1e6,
              "prepare_rest_s": c.get("prepare_rest_us", 0) / 1e6}
    return {"value": m["windows_total"] / t, "unit": "k-mers/s", "upload_prepare_s": prep_s,
            "step_s": m["ms_per_step"] / 1000.0, "phases": phases,
            "note": "host arrays -> HBM (skm_build_add_batch: pinned double-buffered staging, packed on the "
                    "host pool) + prepare + one step"}


def _annotate_leg(skm, kept, funcs, q, a, device, cores):
    """kmers-call-functions path (BASELINE configs[3]): 10M fresh query proteins of the same
    families (genome files after the C2 training set: their own RNG streams) against the CMPH/BDZ
    DB of the C2 build, resident in HBM.  One step = window lookup (k_lookup) + HitSet calls +
    compaction over every query; the calls stay on the device.  Roofline: k_lookup<0>, SURVEY
    8(d) B_alg = 1 B/residue + 18 B/window."""
    import tempfile
    res, off, lens, _, _ = q.packed()
    with tempfile.TemporaryDirectory(dir="/tmp") as d:
        base = os.path.join(d, "kmer_data")
        t0 = time.time()
        skm.mph_build(kept.keys, kept.data, base + ".mph", base + ".dat", seed=1, device=device)
        mph_s = time.time() - t0
        db = skm.CmphKmerDb(base, device=device)
        files = None if a.no_cpu_baseline else (open(base + ".mph", "rb").read(), open(base + ".dat", "rb").read())
    hypo = funcs.index("hypothetical protein")
    qb = skm.QueryBatch(db, res, off, lens)
    nwin = _windows(lens)
    for _ in range(max(1, a.warmup)):
        qb.run(hypo)
    steps = max(3, min(a.steps, 10))
    acc = {}
    t1 = time.perf_counter()
    for _ in range(steps):
        qb.run(hypo)
        for k, v in qb.timings().items():
            acc[k] = acc.get(k, 0.0) + v
    wall = time.perf_counter() - t1
    acc = {k: v / steps for k, v in acc.items()}
    _, calls = qb.calls()
    qb.close()
    db.close()
    alg = int(len(res)) + 18 * nwin
    gbs = alg / (acc["lookup"] * 1e-3) / 1e9
    cpu = None
    if files is not None:  # the call path of the oracle on the host cores, bounded sample
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_ref
        threads = a.cpu_threads or cores["usable"]
        n = min(len(lens), 200_000)
        end = int(off[n - 1]) + int(lens[n - 1])
        ob = oracle_ref.Bdz(files[0])
        t = time.perf_counter()
        oracle_ref.annotate_mt(ob, files[1], res[:end], off[:n], lens[:n], threads, hypo_index=hypo)
        dt = time.perf_counter() - t
        w = _windows(lens[:n])
        cpu = {"value": w / dt, "unit": "k-mers/s", "cores": threads, "kind": "port",
               "host": {k: cores[k] for k in ("model", "affinity", "cgroup_quota")},
               "sample": f"first {n} query proteins ({w} windows), {dt:.1f} s, oracle/skm_oracle.cpp "
                         f"oracle_annotate_mt (process_aa_seq per sequence) on {threads} host threads"}
        del ob, files
    return {"metric": "query k-mers/sec (window lookup + HitSet calls)", "value": nwin * steps / wall,
            "unit": "k-mers/s", "ms_per_step": 1000.0 * wall / steps, "steps": steps,
            "config": {"workload": f"C4: {len(lens):,} fresh query proteins of the same families vs the CMPH DB "
                                   f"of the C2 build in HBM, 1 GPU", "queries": int(len(lens)),
                       "windows": nwin, "db_keys": int(len(kept.keys)), "calls": int(len(calls))},
            "phase_ms": acc,
            "roofline": {"bound": "hbm", "kernel": "k_lookup<0>", "achieved": gbs, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS, "alg_bytes_per_launch": alg,
                         "avg_launch_ms": acc["lookup"], "traffic": _pmc_traffic("k_lookup<0>", "legs", len(lens))},
            "cpu_baseline": cpu, "mph_build_s": mph_s}


def _recall_leg(skm, kept, funcs, train, a, device, cores):
    """The recall pass (kmers-build-signatures.cc:238-349): the C2 training proteins
    called against the exact kept-k-mer DB of their own build (KeptKmerDB, kept_kmer_db.h:20-27;
    the device open-addressing key table), resident in HBM.  One step = window lookup in the exact
    table + HitSet calls over every training protein; the calls stay on the device.  Roofline:
    k_lookup<LK_EXACT>, B_alg = 1 B/residue + 18 B/window (the 8-byte key compared + the 10-byte
    record, as SURVEY 8(d) prices a lookup).  CPU baseline: the oracle's process_aa_seq against the
    sorted kept set (oracle_annotate_exact) on the host cores, bounded sample."""
    res, off, lens, _, _ = train.packed()
    t0 = time.time()
    db = skm.KeptKmerDb(kept.keys, kept.data, device=device)
    open_s = time.time() - t0
    hypo = funcs.index("hypothetical protein")
    qb = skm.QueryBatch(db, res, off, lens)
    nwin = _windows(lens)
    for _ in range(max(1, a.warmup)):
        qb.run(hypo)
    steps = max(3, min(a.steps, 10))
    acc = {}
    t1 = time.perf_counter()
    for _ in range(steps):
        qb.run(hypo)
        for k, v in qb.timings().items():
            acc[k] = acc.get(k, 0.0) + v
    wall = time.perf_counter() - t1
    acc = {k: v / steps for k, v in acc.items()}
    _, calls = qb.calls()
    qb.close()
    db.close()
    alg = int(len(res)) + 18 * nwin
    gbs = alg / (acc["lookup"] * 1e-3) / 1e9
    cpu = None
    if not a.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_ref
        threads = a.cpu_threads or cores["usable"]
        n = min(len(lens), 200_000)
        end = int(off[n - 1]) + int(lens[n - 1])
        t = time.perf_counter()
        _, oc = oracle_ref.annotate_exact_par(kept.keys, kept.data, res[:end], off[:n], lens[:n], threads,
                                              hypo_index=hypo)
        dt = time.perf_counter() - t
        w = _windows(lens[:n])
        cpu = {"value": w / dt, "unit": "k-mers/s", "cores": threads, "kind": "port",
               "host": {k: cores[k] for k in ("model", "affinity", "cgroup_quota")},
               "sample": f"first {n} training proteins ({w} windows), {dt:.1f} s, oracle/skm_oracle.cpp "
                         f"oracle_annotate_exact (process_aa_seq vs the sorted kept set) on {threads} host threads"}
    return {"metric": "training k-mers/sec (recall: exact-DB window lookup + HitSet calls)",
            "value": nwin * steps / wall, "unit": "k-mers/s", "ms_per_step": 1000.0 * wall / steps, "steps": steps,
            "config": {"workload": f"recall: the {len(lens):,} C2 training proteins vs the exact DB of their own "
                                   f"build ({len(kept.keys):,} kept k-mers) in HBM, 1 GPU",
                       "proteins": int(len(lens)), "windows": nwin, "db_keys": int(len(kept.keys)),
                       "calls": int(len(calls))},
            "phase_ms": acc,
            "roofline": {"bound": "hbm", "kernel": "k_lookup<LK_EXACT>", "achieved": gbs, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS, "alg_bytes_per_launch": alg,
                         "avg_launch_ms": acc["lookup"], "traffic": _pmc_traffic("k_lookup<1>", "legs", 10_000_000 if len(lens) == 1_000_000 else -1)},
            "cpu_baseline": cpu, "db_open_s": open_s}


def _matrix_leg(skm, matrix_in, a, device, cores, rank=0, world=1, dist=None):
    """kmers-matrix-distance (BASELINE configs[4]): a 200-family signature DB (built on this GPU from
    200K training proteins, BDZ on the GPU) resident in HBM, 100K fresh query proteins of the same
    families, all-vs-all shared-signature-k-mer counts.  With N ranks each GPU looks up its own
    range of the queries, the hits go to their k-mer's owner (all-to-all), each owner groups its
    k-mers and routes every group's member suffix to the row bands it touches (skm_matrix_tile_rows,
    equal triangle area; all-to-all), each rank counts its band, and the step time is the max over
    ranks.  One step =
    window lookup + length filter, k-mer grouping (hash + radix sort), per-row LDS histograms of the
    pair increments, compaction of the nonzero pairs in row order; the pairs stay on the device.
    Roofline: k_md_rows (the pair increments), SURVEY 8(d) 4 B per pair increment."""
    import tempfile
    train, qs, funcs = matrix_in
    t0 = time.time()
    b = skm.SignatureBuilder(len(funcs), device=device)
    train.add_to(b)
    kept = b.finish()
    b.close()
    res, off, ln, _, _ = qs.packed()
    n = min(a.matrix_seqs, len(ln))
    end = int(off[n - 1]) + int(ln[n - 1])
    res, off, ln = res[:end], off[:n], ln[:n]
    with tempfile.TemporaryDirectory(dir="/tmp") as d:
        base = os.path.join(d, "kmer_data")
        skm.mph_build(kept.keys, kept.data, base + ".mph", base + ".dat", seed=1, device=device)
        db = skm.CmphKmerDb(base, device=device)
        files = None if a.no_cpu_baseline else (open(base + ".mph", "rb").read(), open(base + ".dat", "rb").read())
    prep_s = time.time() - t0
    if world > 1:  # rank r: its contiguous range of the queries; hits to k-mer owners, groups to row bands
        part = np.array_split(np.arange(n), world)[rank]
        qa, qb = (int(part[0]), int(part[-1]) + 1) if len(part) else (0, 0)
        md = skm.MatrixDistance(db, funcs, res, off[qa:qb], ln[qa:qb], seq_idx=np.arange(qa, qb, dtype=np.uint32),
                                n_idx=n)
        if a.comm == "host":
            md.set_transport(skm.GlooTransport())
        else:
            box = [skm.comm_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(box, src=0)
            md.set_comm(box[0], rank, world)
    else:
        md = skm.MatrixDistance(db, funcs, res, off, ln)
    rows = None
    for _ in range(max(1, a.warmup)):
        md.run(rows)
    steps = max(3, min(a.steps, 10))
    acc = {}
    if dist is not None:
        dist.barrier()
    t1 = time.perf_counter()
    for _ in range(steps):
        md.run(rows)
        for k, v in md.timings().items():
            acc[k] = acc.get(k, 0.0) + v
    wall = time.perf_counter() - t1
    acc = {k: v / steps for k, v in acc.items()}
    c = md.counters()
    if dist is not None:  # max time over ranks; pair work summed over the bands
        import torch
        dist.barrier()
        tt = torch.tensor([wall], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        wall = float(tt.item())
        v = torch.tensor([float(c["increments"]), float(c["pairs"]), float(c["windows"]), float(c["local_hits"])],
                         dtype=torch.float64)
        dist.all_reduce(v, op=dist.ReduceOp.SUM)
        c = dict(c, increments=int(v[0]), pairs=int(v[1]), windows=int(v[2]), hits=int(v[3]))
    md.close()
    db.close()
    alg = 4 * c["increments"]
    gbs = alg / (acc["pairs"] * 1e-3) / 1e9
    split = ("query ranges per GPU, hits owner-partitioned by k-mer, k-mer groups routed to the row bands of the "
             "triangle" if world > 1 else "one tile")
    cpu = None
    if files is not None and world == 1:  # the oracle's matrix distance on the host cores, bounded sample
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_ref
        threads = a.cpu_threads or cores["usable"]
        ns = n
        e2 = int(off[ns - 1]) + int(ln[ns - 1])
        ob = oracle_ref.Bdz(files[0])
        t = time.perf_counter()
        oracle_ref.matrix_distance_mt(ob, files[1], res[:e2], off[:ns], ln[:ns], np.arange(ns, dtype=np.uint32),
                                      funcs.index("hypothetical protein"), n_threads=threads, want_pairs=False)
        dt = time.perf_counter() - t
        w = _windows(ln[:ns])
        cpu = {"value": w / dt, "unit": "k-mers/s", "cores": threads, "kind": "port",
               "host": {k: cores[k] for k in ("model", "affinity", "cgroup_quota")},
               "sample": f"all-vs-all over the {ns} query proteins ({w} windows, "
                         f"{dt:.1f} s: the whole C5 workload, measured, not extrapolated), "
                         f"oracle/skm_oracle.cpp oracle_matrix_distance on {threads} host threads"}
        del ob, files
    return {"metric": "query k-mers/sec (lookup + all-vs-all shared signature k-mer counts)",
            "value": c["windows"] * steps / wall, "unit": "k-mers/s", "ms_per_step": 1000.0 * wall / steps,
            "steps": steps, "pair_increments_per_s": c["increments"] / (acc["pairs"] * 1e-3),
            "scaling": "strong", "n_gpus": world,
            "config": {"workload": f"C5: {n} query proteins of 200 families, all-vs-all, {world} GPU(s) ({split})",
                       "queries": n, "families": 200, "db_keys": int(len(kept.keys)), "windows": c["windows"],
                       "hits": c["hits"], "pair_increments": c["increments"], "nonzero_pairs": c["pairs"]},
            "phase_ms": acc,
            "roofline": {"bound": "hbm", "kernel": "k_md_rows", "achieved": gbs, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS, "alg_bytes_per_launch": alg,
                         "avg_launch_ms": acc["pairs"], "traffic": _pmc_traffic("k_md_rows", "legs", 10_000_000 if n == 100_000 else -1)},
            "cpu_baseline": cpu, "prep_s": prep_s}


def _per_launch(traffic, passes):
    return None if traffic is None else traffic / max(1, passes)


_PMC_FILE = "r06_pmc_traffic.json"


def src_sha16() -> str:
    """Hash of libskm's device sources (signature_kmers_amd/csrc/*.hip, *.h): a PMC profile counts
    for the benched code only if it was taken on the same sources."""
    import glob
    import hashlib
    h = hashlib.sha256()
    d = os.path.join(ROOT, "signature_kmers_amd", "csrc")
    for f in sorted(glob.glob(os.path.join(d, "*.hip")) + glob.glob(os.path.join(d, "*.h"))):
        h.update(os.path.basename(f).encode())
        h.update(open(f, "rb").read())
    return h.hexdigest()[:16]


def _pmc_traffic(kernel: str, workload: str, seqs: int):
    """HBM bytes of `kernel` from the committed rocprofv3 PMC summary (profiles/r06_pmc_traffic.json,
    tools/gpu_profile.sh + tools/pmc_summary.py): per build run (all launches of a step)
    or per launch (legs), when it was measured on this kernel and workload size AND on the same
    device sources as this run (src_sha16); else None.  Streaming kernels count FETCH_SIZE x2,
    gather kernels x1 (profiles/r02_fetch_calib.json)."""
    path = os.path.join(ROOT, "profiles", _PMC_FILE)
    try:
        d = json.load(open(path))
        if d.get("src_sha16") != src_sha16():
            return None
        wl = d["workloads"][workload]
        if int(wl.get("seqs", wl.get("queries", -1))) != int(seqs):
            return None
        return d["kernels"][kernel][workload]["hbm_bytes"]
    except Exception:
        return None


def _cpu_baseline(shard, nfun, n_sample, threads, cores, what):
    """The CPU port of the build (oracle/skm_oracle.cpp oracle_build_mt: the --n-threads 1 results
    computed on every usable host core -- extract into key-hash shards, per-shard stable sort +
    group + cut + statistics) on the first n_sample sequences of the workload (`what` says which)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ref
    nf = (n_sample + PER_FILE - 1) // PER_FILE
    r, o, l, f, i = shard.packed(first_files=nf)
    n = min(n_sample, len(l))
    end = int(o[n - 1]) + int(l[n - 1])
    t = time.perf_counter()
    oracle_ref.build_mt(r[:end], o[:n], l[:n], f[:n], i[:n], nfun, threads, sort=False)
    dt = time.perf_counter() - t
    w = oracle_ref.count_windows(l[:n], f[:n])
    return {"value": w / dt, "unit": "k-mers/s", "cores": threads, "kind": "port",
            "host": {k: cores[k] for k in ("model", "affinity", "cgroup_quota")},
            "sample": f"{what}: {w:,} windows in {dt:.1f} s, oracle/skm_oracle.cpp oracle_build_mt on {threads} "
                      f"host threads (every CPU of this job's cgroup quota; --n-threads 1 results, unsorted output "
                      f"like the reference's hash map)"}


if __name__ == "__main__":
    main()
