"""Edge-case input directories for the CLI front end (FASTA dialects, SEED assignment rules).

Covers what function_map.h / fasta_parser.h / signature_build.tcc make observable: id
assignments from definition files (with '#' comments, truncation comments, later files
overriding earlier ones), deflines with "[genome]" suffixes, fig ids, files whose genome falls
back to the file name, deleted features, good functions / good roles / ignored functions,
min-reps, CR line endings, lower case, bad characters, '*' at the start of a continuation line,
empty files and leading garbage.  Deterministic (seeded).
"""
from __future__ import annotations

import os

import numpy as np

AA = b"ACDEFGHIKLMNPQRSTVWY"


def _seq(rng, n, anc=None, sub=0.1):
    if anc is None:
        return bytes(rng.choice(list(AA), size=n).astype(np.uint8))
    a = np.frombuffer(anc, np.uint8).copy()
    m = rng.random(len(a)) < sub
    a[m] = rng.choice(list(AA), size=int(m.sum()))
    return bytes(a)


def _wrap(s: bytes, w=60, crlf=False):
    nl = b"\r\n" if crlf else b"\n"
    return b"".join(s[i:i + w] + nl for i in range(0, len(s), w))


def write_edge_dirs(root: str, seed: int = 7, n_genomes: int = 6, per_genome: int = 40):
    rng = np.random.default_rng(seed)
    defs = os.path.join(root, "defs")
    seqs = os.path.join(root, "Seqs")
    keep = os.path.join(root, "Keep")
    for d in (defs, seqs, keep):
        os.makedirs(d, exist_ok=True)
    funcs = [b"alpha protein", b"beta synthase / gamma kinase", b"delta reductase; epsilon oxidase",
             b"zeta transporter @ eta permease", b"theta factor", b"iota rare", b"kappa good",
             b"hypothetical protein", b"lambda ignored", b"mu fragmentish"]
    anc = {f: _seq(rng, int(rng.integers(60, 240))) for f in funcs}
    def_lines = []
    override_lines = []
    deleted = []
    for g in range(n_genomes):
        gname = f"{1000 + g}.1"
        fname = gname if g != 3 else f"genome_file_{g}"  # g=3: genome from [..] / file name
        crlf = g == 2
        parts = []
        if g == 4:
            parts.append(b"junk before the first header\n")
        for k in range(per_genome):
            pid = f"fig|{gname}.peg.{k + 1}".encode()
            f = funcs[int(rng.integers(0, len(funcs)))]
            if f == b"iota rare" and g > 0:
                f = b"alpha protein"  # iota appears in one genome only (fails min-reps)
            s = _seq(rng, len(anc[f]) + int(rng.integers(-5, 6)) if len(anc[f]) > 10 else 20, None)
            s = _seq(rng, 0, anc[f][:max(10, len(anc[f]) + int(rng.integers(-5, 1)))])
            if rng.random() < 0.05:
                s = s[:5]  # shorter than k
            if g == 1 and k % 7 == 0:
                s = s.lower()
            hdr = b">" + pid
            r = rng.random()
            if g == 3 or r < 0.15:
                # defline with function and [genome]
                ff = f + (b" # some comment" if rng.random() < 0.3 else b"")
                if rng.random() < 0.1:
                    ff = f + b" ## truncated at end"
                hdr += b"  " + ff + b" [Genus species " + gname.encode() + b"]"
            elif r < 0.25:
                hdr += b"\t" + f  # defline without [genome]: whole def is the function
            else:
                c = b""
                if rng.random() < 0.1:
                    c = b" # fragment of something"
                elif rng.random() < 0.1:
                    c = b" # note"
                if rng.random() < 0.9:
                    def_lines.append(pid + b"\t" + f + c + (b"\textra col" if rng.random() < 0.2 else b""))
                if rng.random() < 0.05:
                    override_lines.append(pid + b"\t" + funcs[int(rng.integers(0, len(funcs)))])
            if rng.random() < 0.04:
                deleted.append(pid)
            body = _wrap(s, 60, crlf)
            if g == 5 and k == 3:
                body = body + b"*MKV\n"  # '*' at the start of a continuation line is dropped
            if g == 5 and k == 4:
                body = b"MK1V-Q\n" + body  # bad characters are dropped
            parts.append(hdr + (b"\r\n" if crlf else b"\n") + body)
        target = keep if g == n_genomes - 1 else seqs
        with open(os.path.join(target, fname), "wb") as fh:
            fh.write(b"".join(parts))
    open(os.path.join(seqs, "empty_file"), "wb").close()
    with open(os.path.join(defs, "a_assign.tsv"), "wb") as fh:
        fh.write(b"\n".join(def_lines) + b"\nbadline-without-tab\n")
    with open(os.path.join(defs, "b_override.tsv"), "wb") as fh:
        fh.write(b"\n".join(override_lines) + b"\n")
    files = {}
    files["good_functions"] = os.path.join(root, "good_functions")
    with open(files["good_functions"], "wb") as fh:
        fh.write(b"iota rare\n")
    files["good_roles"] = os.path.join(root, "good_roles")
    with open(files["good_roles"], "wb") as fh:
        fh.write(b"eta permease\n\n")
    files["deleted"] = os.path.join(root, "deleted")
    with open(files["deleted"], "wb") as fh:
        fh.write(b"\n".join(deleted) + b"\n")
    files["ignored"] = os.path.join(root, "ignored")
    with open(files["ignored"], "wb") as fh:
        fh.write(b"lambda ignored\n")
    return dict(defs=defs, seqs=seqs, keep=keep, **files)


def front_args(d, min_reps=2):
    return ["-D", d["defs"], "-F", d["seqs"], "-K", d["keep"], "--good-functions", d["good_functions"],
            "--good-roles", d["good_roles"], "--deleted-features-file", d["deleted"],
            "--ignored-functions-file", d["ignored"], "--min-reps-required", str(min_reps)]


def read_set(path):
    with open(path, "rb") as fh:
        lines = fh.read().split(b"\n")
    if lines and lines[-1] == b"":
        lines.pop()
    return lines
