"""Round-4 diagnosis (GPU box): the CLI's .sai for r100.default with the GPU parse, the host parse and
the golden; the engine path (no CLI) on the same reads; the first differing read of each."""
import os, subprocess, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import oracle
from ibwa_amd import engine as E
G = os.path.join(ROOT, "tests", "golden")
CLI = os.path.join(ROOT, "ibwa_amd", "bin", "ibwa-amd")

def recs(b):
    d = np.frombuffer(b, dtype=np.uint8); p, out = 64, []
    while p < len(d):
        k = int(d[p:p + 4].view(np.int32)[0]); out.append(d[p + 4:p + 4 + 16 * k].tobytes()); p += 4 + 16 * k
    return out

def first_diff(a, b):
    for i, (x, y) in enumerate(zip(a, b)):
        if x != y: return i, len(x) // 16, len(y) // 16
    return (None if len(a) == len(b) else min(len(a), len(b))), len(a), len(b)

key = sys.argv[1] if len(sys.argv) > 1 else "r100.default"
import json
m = json.load(open(os.path.join(G, "sai_manifest.json")))[key]
gold = recs(open(os.path.join(G, key + ".sai"), "rb").read())
for name, env in (("gpu-parse", {}), ("host-parse", {"IBWA_ALN_GPU_PARSE": "0"}), ("serial", {"IBWA_ALN_SERIAL_READ": "1"})):
    out = "/tmp/d.sai"
    r = subprocess.run([CLI, "aln"] + m["argv"] + ["-f", out, os.path.join(G, "g1m"), os.path.join(G, m["reads"])],
                       capture_output=True, text=True, env=dict(os.environ, **env))
    got = recs(open(out, "rb").read())
    print(name, "rc", r.returncode, "reads", len(got), "gold", len(gold), "first diff", first_diff(got, gold), flush=True)
    if r.returncode: print(r.stderr[-800:])
eng = E.Engine(0)
eng.load_index_files(os.path.join(G, "g1m"))
opt, _ = oracle.parse_aln_args(m["argv"])
rr = oracle.read_fastq_records(os.path.join(G, m["reads"]))
seqs, offs, lens = oracle.encode_reads(rr, opt.mode, opt.trim_qual)
e = E.GapOpt()
for f, _ in E.GapOpt._fields_: setattr(e, f, getattr(opt, f))
for tune in ({}, {"gap_lw": 0}, {"gap_resume": 0}, {"gapped_v2": 0}):
    for k, v in tune.items(): eng.set_option(k, v)
    n_aln, alns = eng.aln(seqs, offs, lens, e)
    got = recs(oracle.sai_bytes(opt, n_aln, alns))
    st = eng.stats()
    print("engine", tune, "first diff", first_diff(got, gold), "path", st.path, "heavy", st.n_heavy, "resumed", st.n_resumed, flush=True)
    for k in tune: eng.set_option(k, {"gap_lw": 1, "gap_resume": 1, "gapped_v2": 1}[k])
