"""Deterministic synthetic proteome generator.

The reference builds from SEED genome exports (scripts/kmers-setup-build.pl:71: Seqs/<genome>
FASTA + Annotations/0/<genome> TSV).  No such data exists offline, so this module generates
protein families with the same directory layout and id conventions:

* F function families named ``function %05d``; ~2 % fusion families ``A / B`` whose ancestor is
  the concatenation of the two parts' ancestors; one ``hypothetical protein`` family of unrelated
  random sequences.
* Ancestor length ~ U{100..560}; residues iid from the UniProt background composition.
* Each sequence picks a family by Zipf(s=1) and copies its ancestor with per-site substitution
  0.20, insertion 0.005 and deletion 0.005; 0.1 % 'X' sites; a trailing '*' on 30 % of sequences.
  ``extras=True`` (the 1K config) adds 0.5 % lower-case residues and a few B/Z/U.
* 3 % label noise: the annotation names a random other family (exercises the 80 % cut).
* Genomes are files of ``per_file`` sequences; one RNG stream per file index, so a shard of
  files is identical whichever process generates it.

``generate_arrays`` returns packed arrays for the C-ABI; ``write_dirs`` writes the FASTA /
annotation directories the reference CLIs consume.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import numpy as np

SEED = 20241115
AA = np.frombuffer(b"ARNDCQEGHILKMFPSTWYV", dtype=np.uint8)
AA_FREQ = np.array([8.25, 5.53, 4.06, 5.45, 1.37, 3.93, 6.75, 7.07, 2.27, 5.96,
                    9.66, 5.84, 2.42, 3.86, 4.70, 6.56, 5.34, 1.08, 2.92, 6.87])
AA_FREQ = AA_FREQ / AA_FREQ.sum()
HYPO = "hypothetical protein"
# 4096-entry sampling table with the background composition (quantised to 1/4096)
_AA_TABLE = np.repeat(AA, np.diff(np.round(np.concatenate([[0.0], np.cumsum(AA_FREQ)]) * 4096).astype(np.int64)))


def _aa(rng, n: int) -> np.ndarray:
    return _AA_TABLE[rng.integers(0, len(_AA_TABLE), size=n)]


@dataclass
class Families:
    names: list            # family name per family id
    anc: np.ndarray        # concatenated ancestor residues (u8)
    anc_off: np.ndarray    # [F+1]
    zipf_p: np.ndarray     # selection probability per family
    hypo_id: int


def make_families(n_families: int, seed: int = SEED) -> Families:
    rng = np.random.default_rng([seed, 0xA11CE])
    n_fusion = max(0, int(round(0.02 * n_families)))
    n_plain = n_families - n_fusion - 1
    names = [f"function {i:05d}" for i in range(n_plain)]
    lens = rng.integers(100, 561, size=n_plain)
    anc_parts = [_aa(rng, int(n)) for n in lens]
    for j in range(n_fusion):
        a, b = (int(x) for x in rng.choice(n_plain, size=2, replace=False))
        names.append(f"{names[a]} / {names[b]}")
        anc_parts.append(np.concatenate([anc_parts[a], anc_parts[b]]))
    names.append(HYPO)
    anc_parts.append(np.zeros(0, dtype=np.uint8))  # hypothetical: unrelated random sequences
    hypo_id = len(names) - 1
    anc_off = np.zeros(len(anc_parts) + 1, dtype=np.int64)
    anc_off[1:] = np.cumsum([len(p) for p in anc_parts])
    anc = np.concatenate(anc_parts).astype(np.uint8)
    ranks = rng.permutation(len(names)) + 1          # Zipf rank of each family
    p = 1.0 / ranks
    return Families(names, anc, anc_off, p / p.sum(), hypo_id)


def _mutate_file(fam: Families, n: int, file_idx: int, seed: int, extras: bool):
    """Members of one genome file.  Returns (residues u8, lens i64, family ids, label ids)."""
    rng = np.random.default_rng([seed, 7, file_idx])
    F = len(fam.names)
    fids = rng.choice(F, size=n, p=fam.zipf_p)
    anc_len = (fam.anc_off[1:] - fam.anc_off[:-1])[fids]
    is_hypo = fids == fam.hypo_id
    anc_len = np.where(is_hypo, rng.integers(100, 561, size=n), anc_len)
    total = int(anc_len.sum())
    seq_start = np.zeros(n + 1, dtype=np.int64)
    seq_start[1:] = np.cumsum(anc_len)
    within = np.arange(total, dtype=np.int64) - np.repeat(seq_start[:-1], anc_len)
    src = np.repeat(fam.anc_off[:-1][fids], anc_len) + within
    hypo_pos = np.repeat(is_hypo, anc_len)
    base = np.empty(total, dtype=np.uint8)
    base[~hypo_pos] = fam.anc[src[~hypo_pos]]
    base[hypo_pos] = _aa(rng, int(hypo_pos.sum()))
    # substitutions (ancestor-derived residues only)
    sub = (rng.random(total) < 0.20) & ~hypo_pos
    base[sub] = _aa(rng, int(sub.sum()))
    # indels: each ancestral slot emits [residue unless deleted][insert if inserted]
    keep = rng.random(total) >= 0.005
    ins = (rng.random(total) < 0.005) & ~hypo_pos
    star = rng.random(n) < 0.30
    # slots: 2 per site, plus one '*' slot at the end of each sequence
    slot_val = np.empty((total, 2), dtype=np.uint8)
    slot_val[:, 0] = base
    slot_val[:, 1] = 0
    slot_val[ins, 1] = _aa(rng, int(ins.sum()))
    slot_ok = np.stack([keep, ins], axis=1)
    per_seq_sites = np.add.reduceat(keep.astype(np.int64) + ins, seq_start[:-1]) if total else np.zeros(n, np.int64)
    per_seq_sites = np.where(anc_len > 0, per_seq_sites, 0)
    out_len = per_seq_sites + star.astype(np.int64)
    flat_vals = slot_val.reshape(-1)[slot_ok.reshape(-1)]
    # insert '*' after each starred sequence
    res = np.empty(int(out_len.sum()), dtype=np.uint8)
    out_start = np.zeros(n + 1, dtype=np.int64)
    out_start[1:] = np.cumsum(out_len)
    site_start = np.zeros(n + 1, dtype=np.int64)
    site_start[1:] = np.cumsum(per_seq_sites)
    dst_idx = np.arange(len(flat_vals), dtype=np.int64)
    seq_of = np.repeat(np.arange(n), per_seq_sites)
    dst_idx = dst_idx - site_start[seq_of] + out_start[seq_of]
    res[dst_idx] = flat_vals
    res[out_start[1:][star] - 1] = ord("*")
    # X sites (not on the trailing '*')
    xs = rng.random(len(res)) < 0.001
    xs[out_start[1:][star] - 1] = False
    res[xs] = ord("X")
    if extras:
        low = rng.random(len(res)) < 0.005
        low &= res != ord("*")
        res[low] = res[low] + 32
        odd = rng.random(len(res)) < 0.0005
        odd &= res != ord("*")
        res[odd] = rng.choice(np.frombuffer(b"BZU", dtype=np.uint8), size=int(odd.sum()))
    # label noise: 3 % annotated with another family
    labels = fids.copy()
    noisy = rng.random(n) < 0.03
    shift = rng.integers(1, F, size=n)
    labels[noisy] = (fids[noisy] + shift[noisy]) % F
    return res, out_len, fids, labels


@dataclass
class Proteome:
    residues: np.ndarray   # u8, sequences back to back
    seq_off: np.ndarray    # u64
    seq_len: np.ndarray    # u32
    labels: np.ndarray     # family id named by the annotation
    file_of: np.ndarray    # genome file index per sequence
    names: list            # family names
    per_file: int
    first_file: int


def generate_arrays(n_seqs: int, n_families: int, per_file: int = 4000, first_file: int = 0,
                    n_files: int | None = None, seed: int = SEED, extras: bool = False) -> Proteome:
    """Sequences of files [first_file, first_file+n_files) of an n_seqs proteome."""
    fam = make_families(n_families, seed)
    total_files = (n_seqs + per_file - 1) // per_file
    if n_files is None:
        n_files = total_files - first_file
    res_parts, len_parts, lab_parts, file_parts = [], [], [], []
    for f in range(first_file, min(total_files, first_file + n_files)):
        n = min(per_file, n_seqs - f * per_file)
        r, L, _, lab = _mutate_file(fam, n, f, seed, extras)
        res_parts.append(r)
        len_parts.append(L)
        lab_parts.append(lab)
        file_parts.append(np.full(n, f, dtype=np.int64))
    residues = np.concatenate(res_parts) if res_parts else np.zeros(0, np.uint8)
    lens = np.concatenate(len_parts).astype(np.uint32) if len_parts else np.zeros(0, np.uint32)
    off = np.zeros(len(lens), dtype=np.uint64)
    if len(lens):
        off[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    return Proteome(residues, off, lens, np.concatenate(lab_parts) if lab_parts else np.zeros(0, np.int64),
                    np.concatenate(file_parts) if file_parts else np.zeros(0, np.int64), fam.names, per_file, first_file)


def function_index_of(names: list) -> dict:
    """FunctionIndex assignment when every family is kept: byte-lexicographic order of the
    function strings with "hypothetical protein" always present (function_map.h:309-330)."""
    kept = sorted(set(names) | {HYPO}, key=lambda s: s.encode())
    return {f: i for i, f in enumerate(kept)}


def build_inputs(p: Proteome):
    """(residues, seq_off, seq_len, seq_func u16, seq_id u32, function list) for skm_build_add_batch,
    with every family kept and seq_id = file_number*100000 + k (signature_build.tcc:91,138)."""
    fi = function_index_of(p.names)
    func_of_family = np.array([fi[n] for n in p.names], dtype=np.uint16)
    seq_func = func_of_family[p.labels]
    # k counts sequences with a non-empty assignment within each file (all of them here)
    file_rel = np.arange(len(p.file_of)) - np.searchsorted(p.file_of, p.file_of, side="left")
    seq_id = (p.file_of * 100000 + file_rel).astype(np.uint32)
    funcs = sorted(fi, key=fi.get)
    return p.residues, p.seq_off, p.seq_len, seq_func, seq_id, funcs


def write_dirs(root: str, n_seqs: int, n_families: int, per_file: int, seed: int = SEED, extras: bool = False,
               genome_base: int = 100000) -> dict:
    """Write ``Seqs/<g>.1`` FASTA (60 columns) and ``Annotations/<g>.1`` TSV (id \\t function)."""
    p = generate_arrays(n_seqs, n_families, per_file, seed=seed, extras=extras)
    seqs_dir = os.path.join(root, "Seqs")
    ann_dir = os.path.join(root, "Annotations")
    os.makedirs(seqs_dir, exist_ok=True)
    os.makedirs(ann_dir, exist_ok=True)
    files = []
    n_files = (n_seqs + per_file - 1) // per_file
    for f in range(n_files):
        g = f"{genome_base + f}.1"
        idx = np.nonzero(p.file_of == f)[0]
        with open(os.path.join(seqs_dir, g), "w") as fa, open(os.path.join(ann_dir, g), "w") as an:
            for k, s in enumerate(idx):
                pid = f"fig|{g}.peg.{k + 1}"
                seq = p.residues[p.seq_off[s]:p.seq_off[s] + p.seq_len[s]].tobytes().decode()
                fa.write(f">{pid}\n")
                for c in range(0, len(seq), 60):
                    fa.write(seq[c:c + 60] + "\n")
                an.write(f"{pid}\t{p.names[p.labels[s]]}\n")
        files.append(g)
    return {"seqs_dir": seqs_dir, "ann_dir": ann_dir, "files": files, "proteome": p}


# ------------------------------------------------------------------------------------------
# Parallel generation (the 50M-protein C3 proteome): files are independent RNG streams, so a
# pool of worker processes generates them in any order and the caller consumes them in file
# order.  Workers are spawned (never forked): the caller may already hold a GPU context.
# ------------------------------------------------------------------------------------------
_WORKER_FAM = {}


def _file_inputs(args):
    """build_inputs of one genome file: (residues, seq_off, seq_len, seq_func, seq_id)."""
    n_seqs, n_families, per_file, f, seed, extras = args
    key = (n_families, seed)
    if key not in _WORKER_FAM:
        fam = make_families(n_families, seed)
        fi = function_index_of(fam.names)
        _WORKER_FAM[key] = (fam, np.array([fi[n] for n in fam.names], dtype=np.uint16))
    fam, func_of_family = _WORKER_FAM[key]
    n = min(per_file, n_seqs - f * per_file)
    res, lens, _, labels = _mutate_file(fam, n, f, seed, extras)
    lens = lens.astype(np.uint32)
    off = np.zeros(n, dtype=np.uint64)
    if n:
        off[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    seq_id = (np.uint32(f) * np.uint32(100000) + np.arange(n, dtype=np.uint32)).astype(np.uint32)
    return res, off, lens, func_of_family[labels], seq_id


def iter_file_inputs(n_seqs: int, n_families: int, per_file: int = 4000, first_file: int = 0,
                     n_files: int | None = None, seed: int = SEED, extras: bool = False, workers: int = 1):
    """Yields build_inputs-style arrays per genome file, in file order, for files
    [first_file, first_file + n_files) of an n_seqs proteome; `workers` > 1 generates them in a
    spawned process pool (identical bytes: one RNG stream per file)."""
    total_files = (n_seqs + per_file - 1) // per_file
    if n_files is None:
        n_files = total_files - first_file
    files = range(first_file, min(total_files, first_file + n_files))
    jobs = [(n_seqs, n_families, per_file, f, seed, extras) for f in files]
    if workers <= 1 or len(jobs) <= 1:
        for j in jobs:
            yield _file_inputs(j)
        return
    import multiprocessing as mp
    with mp.get_context("spawn").Pool(workers) as pool:
        yield from pool.imap(_file_inputs, jobs, chunksize=4)


def functions(n_families: int, seed: int = SEED) -> list:
    """The function list (FunctionIndex order) of a proteome of n_families families."""
    fi = function_index_of(make_families(n_families, seed).names)
    return sorted(fi, key=fi.get)


def fasta_bytes(ids, residues: np.ndarray, lens: np.ndarray, width: int = 60) -> bytes:
    """FASTA text of records (id, residues[off:off+len]) wrapped at `width` columns, as
    write_dirs writes it, built without a per-line Python loop."""
    out = []
    off = 0
    for pid, n in zip(ids, lens.tolist()):
        seq = residues[off:off + n]
        off += n
        out.append(b">" + pid + b"\n")
        if n:
            rows = (n + width - 1) // width
            pad = np.full(rows * (width + 1), 10, np.uint8)
            view = pad.reshape(rows, width + 1)
            full = n // width
            if full:
                view[:full, :width] = seq[:full * width].reshape(full, width)
            rem = n - full * width
            if rem:
                view[full, :rem] = seq[full * width:]
                out.append(pad[:full * (width + 1) + rem + 1].tobytes())
            else:
                out.append(pad.tobytes())
    return b"".join(out)


def _write_file(args):
    """One genome file of write_dirs: Seqs/<g>.1 and Annotations/<g>.1 (identical bytes)."""
    root, n_seqs, n_families, per_file, f, seed, extras, genome_base = args
    key = (n_families, seed)
    if key not in _WORKER_FAM:
        fam = make_families(n_families, seed)
        fi = function_index_of(fam.names)
        _WORKER_FAM[key] = (fam, np.array([fi[n] for n in fam.names], dtype=np.uint16))
    fam, _ = _WORKER_FAM[key]
    n = min(per_file, n_seqs - f * per_file)
    res, lens, _, labels = _mutate_file(fam, n, f, seed, extras)
    g = f"{genome_base + f}.1"
    ids = [f"fig|{g}.peg.{k + 1}".encode() for k in range(n)]
    with open(os.path.join(root, "Seqs", g), "wb") as fa:
        fa.write(fasta_bytes(ids, res, lens.astype(np.int64)))
    with open(os.path.join(root, "Annotations", g), "wb") as an:
        an.write(b"".join(b"%s\t%s\n" % (pid, fam.names[lab].encode()) for pid, lab in zip(ids, labels)))
    return g


def write_dirs_parallel(root: str, n_seqs: int, n_families: int, per_file: int, seed: int = SEED,
                        extras: bool = False, genome_base: int = 100000, workers: int = 8, first_file: int = 0,
                        n_files: int | None = None) -> dict:
    """write_dirs with the files generated and written by a spawned process pool (the same bytes);
    files [first_file, first_file + n_files) of an n_seqs proteome; no in-memory proteome is
    returned (iter_file_inputs regenerates the build arrays)."""
    seqs_dir = os.path.join(root, "Seqs")
    ann_dir = os.path.join(root, "Annotations")
    os.makedirs(seqs_dir, exist_ok=True)
    os.makedirs(ann_dir, exist_ok=True)
    total = (n_seqs + per_file - 1) // per_file
    last = total if n_files is None else min(total, first_file + n_files)
    jobs = [(root, n_seqs, n_families, per_file, f, seed, extras, genome_base) for f in range(first_file, last)]
    if workers <= 1:
        files = [_write_file(j) for j in jobs]
    else:
        import multiprocessing as mp
        with mp.get_context("spawn").Pool(workers) as pool:
            files = list(pool.imap(_write_file, jobs, chunksize=2))
    return {"seqs_dir": seqs_dir, "ann_dir": ann_dir, "files": files}
