#!/usr/bin/env python3
"""Generate tests/golden/pe_*: paired reads, their .sai and the reference's sampe SAM (build container only).

TEST INFRASTRUCTURE.  Mate pairs are drawn from the golden g1m genome (tests/synth_util.py) with
a mix of the situations sampe's code paths branch on: proper pairs, pairs with one end made
unalignable by `aln` but rescuable by bwa_paired_sw (dense mismatches), random (unmappable) ends,
discordant pairs (far apart / same strand / different contigs), pairs inside repeat families,
reads with N, fragments at contig ends and reads with low base qualities (for `aln -q`).
The reference's own `aln` and `sampe` (bwa_sai2sam_pe_core, bwape.c:436-540, compiled into
oracle/_ref/ibwa_ref by oracle/Makefile) are run on them; the FASTQ, .sai and gzip'd SAM are
committed with sampe_manifest.json.  The @PG line names the program that wrote the file and is
not compared.
"""
import gzip
import json
import os
import random
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
REF = os.path.join(ROOT, "oracle", "_ref", "ibwa_ref")
sys.path.insert(0, ROOT)

from tests.synth_util import golden_genome_ascii  # noqa: E402

COMP = str.maketrans("ACGTN", "TGCAN")

# read set -> (read length, insert avg, insert std, substitution rate, pairs, seed)
SETS = {
    "pe100": (100, 300.0, 30.0, 0.01, 1500, 11),
    "pe150": (150, 350.0, 35.0, 0.02, 600, 12),
    "pe70few": (70, 250.0, 20.0, 0.01, 15, 13),  # too few pairs: insert size not inferred
}
# sampe cases: key -> (read set, aln options, sampe options)
CASES = {
    "pe100.default": ("pe100", [], ["-R"]),
    "pe100.noR": ("pe100", [], []),  # without -R the reference unmaps every read (select_sai_ibwa's remap status)
    "pe100.s": ("pe100", [], ["-R", "-s"]),
    "pe100.A": ("pe100", [], ["-R", "-A"]),
    "pe100.a1000": ("pe100", [], ["-R", "-a", "1000"]),
    "pe100.n5N20": ("pe100", [], ["-R", "-n", "5", "-N", "20"]),
    "pe100.n0N0": ("pe100", [], ["-R", "-n", "0", "-N", "0"]),
    "pe100.c1e-3": ("pe100", [], ["-R", "-c", "1e-3"]),
    "pe100.rg": ("pe100", [], ["-R", "-r", "@RG\\tID:lane1\\tSM:x"]),
    "pe100.q20": ("pe100", ["-q", "20"], ["-R"]),
    "pe100.k0n3": ("pe100", ["-k", "0", "-n", "3"], ["-R"]),
    "pe150.default": ("pe150", [], ["-R"]),
    "pe150.o1000": ("pe150", [], ["-R", "-o", "1000"]),
    "pe70few.default": ("pe70few", [], ["-R"]),
    # sampe -t T: thread t pairs t, t+T, ... in its own position array (bwape.c:249-253), so
    # find_optimal_pair's look-ahead reads what the pair's residue class mod T left there
    "pe100.t4": ("pe100", [], ["-R", "-t", "4"]),
}


def rc(s):
    return s.translate(COMP)[::-1]


def mutate(rng, s, sub):
    out = list(s)
    for i in range(len(out)):
        if out[i] != "N" and rng.random() < sub:
            out[i] = rng.choice([b for b in "ACGT" if b != out[i]])
    s = "".join(out)
    if rng.random() < 0.05:  # one short indel
        p = rng.randrange(10, len(s) - 10)
        if rng.random() < 0.5:
            s = (s[:p] + "".join(rng.choice("ACGT") for _ in range(rng.randint(1, 3))) + s[p:])[:len(out)]
        else:
            d = rng.randint(1, 3)
            s = s[:p] + s[p + d:] + "".join(rng.choice("ACGT") for _ in range(d))
    return s


def qual(rng, L, low_tail):
    q = [chr(33 + rng.randint(20, 40)) for _ in range(L)]
    if low_tail:
        for i in range(L - rng.randint(5, 30), L):
            q[i] = chr(33 + rng.randint(2, 12))
    return "".join(q)


def make_pairs(genome, starts, rng, L, avg, std, sub, n):
    G = len(genome)
    kinds = ["pair"] * 6 + ["dense1", "dense2", "rand1", "rand2", "disc", "samestrand", "far", "withN", "edge",
                            "lowq", "repeat"]
    r1s, r2s = [], []
    while len(r1s) < n:
        kind = kinds[len(r1s) % len(kinds)]
        ins = max(L + 10, int(rng.gauss(avg, std)))
        if kind == "edge":
            c = rng.randrange(len(starts) - 1)
            f = rng.choice([starts[c] + rng.randrange(0, 40), starts[c + 1] - ins - rng.randrange(0, 40)])
        else:
            f = rng.randrange(0, G - ins)
        seg = genome[f:f + ins]
        if "N" in seg and kind != "withN":
            continue
        if kind == "withN" and "N" not in seg:
            seg = seg[:ins // 3] + "N" + seg[ins // 3 + 1:]
        a, b = mutate(rng, seg[:L], sub), mutate(rng, rc(seg[-L:]), sub)
        if kind == "dense1":  # aln misses end 1 (9 mismatches), local SW still finds it
            a = mutate(rng, seg[:L], 0.09)
        elif kind == "dense2":
            b = mutate(rng, rc(seg[-L:]), 0.09)
        elif kind == "rand1":
            a = "".join(rng.choice("ACGT") for _ in range(L))
        elif kind == "rand2":
            b = "".join(rng.choice("ACGT") for _ in range(L))
        elif kind == "samestrand":
            b = mutate(rng, seg[-L:], sub)
        elif kind == "far":
            g = rng.randrange(0, G - L)
            if "N" in genome[g:g + L]:
                continue
            b = mutate(rng, rc(genome[g:g + L]), sub)
        elif kind == "disc":
            b = mutate(rng, rc(genome[f + ins + 2000:f + ins + 2000 + L]), sub) if f + ins + 2000 + L < G else b
        if len(a) != L or len(b) != L:
            continue
        if rng.random() < 0.5:  # which end comes first in the fragment
            a, b = b, a
        low = kind == "lowq"
        r1s.append((a, qual(rng, L, low)))
        r2s.append((b, qual(rng, L, low and rng.random() < 0.5)))
    return r1s, r2s


def write_fq(path, name, recs, suffix):
    with open(path, "w") as f:
        for i, (s, q) in enumerate(recs):
            f.write(f"@{name}{i}/{suffix}\n{s}\n+\n{q}\n")


def tandem_case():
    """A 160 kb genome holding a 60 kb tandem array of a 50 bp unit (1 200 exact copies, except every
    100th copy with one substitution) between random sequence, indexed by the reference; pairs from inside the array
    (SA intervals of > 1 000 rows: the bwtcache path, position arrays of thousands of entries sorted
    by the restated introsort with ties across the two ends), pairs across its edges, and
    consecutive duplicate pairs (find_optimal_pair's look-ahead into the previous pair's array)."""
    rng = random.Random(21)
    unit = "".join(rng.choice("ACGT") for _ in range(50))
    arr = []
    for c in range(1200):
        u = list(unit)
        if c % 100 == 99:
            k = rng.randrange(50)
            u[k] = rng.choice([b for b in "ACGT" if b != u[k]])
        arr.append("".join(u))
    left = "".join(rng.choice("ACGT") for _ in range(50000))
    right = "".join(rng.choice("ACGT") for _ in range(50000))
    g = left + "".join(arr) + right
    with open(os.path.join(GOLD, "tandem.fa"), "w") as f:
        f.write(">tr1 tandem array\n")
        for i in range(0, len(g), 70):
            f.write(g[i:i + 70] + "\n")
    subprocess.run([REF, "index", "-p", os.path.join(GOLD, "tandem"), os.path.join(GOLD, "tandem.fa")], check=True,
                   capture_output=True)
    L = 100
    r1s, r2s = [], []
    while len(r1s) < 400:
        ins = max(L + 10, int(rng.gauss(300, 30)))
        kind = len(r1s) % 4
        if kind == 0 or kind == 1:  # inside the array
            f0 = rng.randrange(50000, 50000 + 60000 - ins)
        elif kind == 2:  # across an edge of the array
            f0 = rng.choice([50000 - rng.randrange(0, ins), 110000 - rng.randrange(0, ins)])
        else:  # unique flanks
            f0 = rng.choice([rng.randrange(0, 45000), rng.randrange(112000, len(g) - ins)])
        seg = g[f0:f0 + ins]
        a, b = mutate(rng, seg[:L], 0.01), mutate(rng, rc(seg[-L:]), 0.01)
        if len(a) != L or len(b) != L:
            continue
        if rng.random() < 0.5:
            a, b = b, a
        q = "I" * L
        r1s.append((a, q))
        r2s.append((b, q))
        if rng.random() < 0.15:  # a duplicate pair right after it
            r1s.append((a, q))
            r2s.append((b, q))
    write_fq(os.path.join(GOLD, "tandem_1.fq"), "td_", r1s, 1)
    write_fq(os.path.join(GOLD, "tandem_2.fq"), "td_", r2s, 2)
    prefix = os.path.join(GOLD, "tandem")
    out = {}
    for key, argv in (("tandem.R", ["-R"]), ("tandem.R.n2000", ["-R", "-n", "2000", "-N", "3000"]),
                      ("tandem.R.t2", ["-R", "-t", "2"]), ("tandem.R.t3", ["-R", "-t", "3"])):
        sai = []
        for end in (1, 2):
            fn = f"tandem_{end}.sai"
            subprocess.run([REF, "aln", "-f", os.path.join(GOLD, fn), prefix, os.path.join(GOLD, f"tandem_{end}.fq")],
                           check=True, capture_output=True)
            sai.append(fn)
        res = subprocess.run([REF, "sampe"] + argv + [prefix] + [os.path.join(GOLD, x) for x in sai] +
                             [os.path.join(GOLD, "tandem_1.fq"), os.path.join(GOLD, "tandem_2.fq")],
                             check=True, capture_output=True)
        with open(os.path.join(GOLD, f"sampe_{key}.sam.gz"), "wb") as raw:
            with gzip.GzipFile(fileobj=raw, mode="wb", mtime=0) as f:
                f.write(res.stdout)
        out[key] = {"prefix": "tandem", "sai": sai, "reads": ["tandem_1.fq", "tandem_2.fq"], "aln_argv": [],
                    "argv": argv, "sam": f"sampe_{key}.sam.gz"}
        print(key, len(res.stdout.splitlines()), "lines")
    return out


def tandem_threads_case():
    """`sampe -t T` on the tandem genome: pairs from inside the array, each followed T pairs later (T = 2
    or 3) by a copy of itself, so the reference's thread-local position arrays (thread t pairs t, t+T, ...,
    bwape.c:249-253) hold the copy's own positions past its end, while one shared array would hold the
    pair just before it.  (Measured with the reference: -t 1, -t 2 and -t 3 give the same SAM here,
    because no look-ahead run reaches past a pair's own positions on this genome; the fixture that
    separates them is tools/make_sampe_stale_golden.py.)"""
    rng = random.Random(33)
    prefix = os.path.join(GOLD, "tandem")
    g = "".join(ln.strip() for ln in open(os.path.join(GOLD, "tandem.fa")) if not ln.startswith(">"))
    L = 100
    r1s, r2s = [], []
    while len(r1s) < 600:
        ins = max(L + 10, int(rng.gauss(300, 30)))
        f0 = rng.randrange(50000, 50000 + 60000 - ins) if rng.random() < 0.8 else rng.randrange(0, 45000)
        seg = g[f0:f0 + ins]
        a, b = mutate(rng, seg[:L], 0.01), mutate(rng, rc(seg[-L:]), 0.01)
        if len(a) != L or len(b) != L:
            continue
        if rng.random() < 0.5:
            a, b = b, a
        r1s.append((a, "I" * L))
        r2s.append((b, "I" * L))
        if len(r1s) >= 3 and rng.random() < 0.3:  # the pair T = 2 or 3 before, again
            t = rng.choice([2, 3])
            r1s.append(r1s[-t])
            r2s.append(r2s[-t])
    write_fq(os.path.join(GOLD, "tandemt_1.fq"), "tt_", r1s, 1)
    write_fq(os.path.join(GOLD, "tandemt_2.fq"), "tt_", r2s, 2)
    sai = []
    for end in (1, 2):
        fn = f"tandemt_{end}.sai"
        subprocess.run([REF, "aln", "-f", os.path.join(GOLD, fn), prefix, os.path.join(GOLD, f"tandemt_{end}.fq")],
                       check=True, capture_output=True)
        sai.append(fn)
    out = {}
    for key, argv in (("tandemt.R", ["-R"]), ("tandemt.R.t2", ["-R", "-t", "2"]), ("tandemt.R.t3", ["-R", "-t", "3"])):
        res = subprocess.run([REF, "sampe"] + argv + [prefix] + [os.path.join(GOLD, x) for x in sai] +
                             [os.path.join(GOLD, "tandemt_1.fq"), os.path.join(GOLD, "tandemt_2.fq")],
                             check=True, capture_output=True)
        with open(os.path.join(GOLD, f"sampe_{key}.sam.gz"), "wb") as raw:
            with gzip.GzipFile(fileobj=raw, mode="wb", mtime=0) as f:
                f.write(res.stdout)
        out[key] = {"prefix": "tandem", "sai": sai, "reads": ["tandemt_1.fq", "tandemt_2.fq"], "aln_argv": [],
                    "argv": argv, "sam": f"sampe_{key}.sam.gz"}
        print(key, len(res.stdout.splitlines()), "lines")
    return out


def main():
    genome, names, lens = golden_genome_ascii()
    starts = [0]
    for ln in lens:
        starts.append(starts[-1] + ln)
    for key, (L, avg, std, sub, n, seed) in SETS.items():
        rng = random.Random(seed)
        r1, r2 = make_pairs(genome, starts, rng, L, avg, std, sub, n)
        write_fq(os.path.join(GOLD, f"{key}_1.fq"), key + "_", r1, 1)
        write_fq(os.path.join(GOLD, f"{key}_2.fq"), key + "_", r2, 2)
    manifest = {}
    prefix = os.path.join(GOLD, "g1m")
    for key, (rs, aln_argv, sampe_argv) in CASES.items():
        sai = []
        for end in (1, 2):
            tag = "default" if not aln_argv else "".join(a.strip("-") for a in aln_argv)
            fn = f"{rs}.{tag}_{end}.sai"
            subprocess.run([REF, "aln"] + aln_argv + ["-f", os.path.join(GOLD, fn), prefix,
                                                      os.path.join(GOLD, f"{rs}_{end}.fq")],
                           check=True, capture_output=True)
            sai.append(fn)
        out = subprocess.run([REF, "sampe"] + sampe_argv + [prefix, os.path.join(GOLD, sai[0]), os.path.join(GOLD, sai[1]),
                                                            os.path.join(GOLD, f"{rs}_1.fq"),
                                                            os.path.join(GOLD, f"{rs}_2.fq")],
                             check=True, capture_output=True)
        with open(os.path.join(GOLD, f"sampe_{key}.sam.gz"), "wb") as raw:
            with gzip.GzipFile(fileobj=raw, mode="wb", mtime=0) as f:
                f.write(out.stdout)
        manifest[key] = {"sai": sai, "reads": [f"{rs}_1.fq", f"{rs}_2.fq"], "aln_argv": aln_argv,
                         "argv": sampe_argv, "sam": f"sampe_{key}.sam.gz"}
        print(key, len(out.stdout.splitlines()), "lines")
    manifest.update(tandem_case())
    manifest.update(tandem_threads_case())
    with open(os.path.join(GOLD, "sampe_manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)


if __name__ == "__main__":
    main()
