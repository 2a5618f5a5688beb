#!/usr/bin/env python3
"""Compressed-input rates of `ibwa-amd aln` by gzip shape, on the GPU box.

The bench's GRCh37-sized synthetic genome and index (built on the device, written as .bwt / .rbwt),
N synthetic 100 bp reads written as plain FASTQ and as three gzip shapes by synth.cpp
(ibwa_synth_write_fastq_gz: BGZF, plain members of ~4 MiB, one member; deflate level 1, binned
qualities), then per file the CLI parse-only (IBWA_ALN_PARSE_ONLY: read, inflate, GPU parse, nothing
aligned) and the CLI end to end.  Every .sai must equal the plain file's.
usage: tools/gz_bench.py [--reads 10000000] [--scale 1.0] [--out FILE]"""
import argparse
import ctypes
import json
import os
import re
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

CLI = os.path.join(ROOT, "ibwa_amd", "bin", "ibwa-amd")


def log(*a):
    print("[gz_bench]", *a, file=sys.stderr, flush=True)


def cli(pre, path, sai, env_extra):
    env = dict(os.environ, IBWA_ALN_TIMES="1", **env_extra)
    t = time.perf_counter()
    r = subprocess.run([CLI, "aln", "-f", sai, pre, path], stdout=subprocess.DEVNULL, stderr=subprocess.PIPE,
                       env=env, timeout=900)
    wall = time.perf_counter() - t
    err = r.stderr.decode(errors="replace")
    if r.returncode != 0:
        raise RuntimeError(err[-1500:])
    out = {"wall_s": wall}
    for ln in err.splitlines():
        if "wall s:" in ln:
            out["phases_s"] = {k.strip(): float(v) for k, v in re.findall(r"([a-z][a-z .()]*?) (\d+\.\d+)",
                                                                            ln.split("wall s:", 1)[1])}
        m = re.search(r"inflated on (\d+) host threads: ([\d.]+) GB in ([\d.]+) s", ln)
        if m:
            out["inflate"] = {"threads": int(m.group(1)), "gb": float(m.group(2)), "reader_thread_s": float(m.group(3)),
                              "gb_per_s": float(m.group(2)) / max(float(m.group(3)), 1e-9)}
        m = re.search(r"parse only: (\d+) reads, ([\d.]+) s parsing \(([\d.]+) s after", ln)
        if m:
            out["parse_only"] = {"reads": int(m.group(1)), "wait_s": float(m.group(2)),
                                 "after_first_group_s": float(m.group(3))}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=10_000_000)
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--level", type=int, default=1)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    from ibwa_amd import engine as E
    from ibwa_amd import _native
    L = _native.lib()
    th = bench.host_threads()
    den = 1_000_000
    ascii_, codes, lens, _ = bench.make_genome(int(round(a.scale * den)), den, 37, th)
    d = tempfile.mkdtemp(prefix="ibwa_gz_", dir=os.environ.get("TMPDIR", "/tmp"))
    res = {"reads": a.reads, "read_len": 100, "genome_bp": int(sum(lens)), "deflate_level": a.level, "host_threads": th}
    try:
        pre = os.path.join(d, "g")
        eng = E.Engine(0)
        eng.build_index(codes)
        del codes
        for s_, ext in ((0, ".bwt"), (1, ".rbwt")):
            p_, L2, w = eng.export_bwt(s_)
            with open(pre + ext, "wb") as f:
                np.array([p_] + list(L2), dtype=np.uint32).tofile(f)
                w.astype(np.uint32, copy=False).tofile(f)
        eng.close()
        n = a.reads
        raw = np.empty(n * 100, dtype=np.uint8)
        pos = np.empty(n, dtype=np.uint64)
        strand = np.empty(n, dtype=np.uint8)
        c_lens = (ctypes.c_uint64 * len(lens))(*lens)
        L.ibwa_synth_reads(bench.shard_seed(0, 3), ascii_.ctypes.data, ascii_.size, len(lens), c_lens, n, 100, 0.01,
                           0.05, raw.ctypes.data, pos.ctypes.data, strand.ctypes.data, th)
        del pos, strand
        files = {"plain": os.path.join(d, "r.fq")}
        t = time.perf_counter()
        if L.ibwa_synth_write_fastq(files["plain"].encode(), raw.ctypes.data, 0, n, 100, th) != 0:
            raise RuntimeError("write fastq")
        res["plain_bytes"] = os.path.getsize(files["plain"])
        for kind, name in ((0, "bgzf"), (1, "members"), (2, "single")):
            files[name] = os.path.join(d, f"r.{name}.fq.gz")
            t = time.perf_counter()
            if L.ibwa_synth_write_fastq_gz(files[name].encode(), raw.ctypes.data, 0, n, 100, th, 1, kind, a.level) != 0:
                raise RuntimeError(f"write {name}")
            res[f"{name}_bytes"] = os.path.getsize(files[name])
            log(f"{name}: {res[f'{name}_bytes'] / 1e9:.2f} GB written in {time.perf_counter() - t:.1f} s")
        del raw
        base_sai = None
        for name, path in files.items():
            sai = os.path.join(d, f"{name}.sai")
            po = cli(pre, path, sai, {"IBWA_ALN_PARSE_ONLY": "1", "IBWA_ARENA_GB": "0"})
            full = cli(pre, path, sai, {})
            ph = full.get("phases_s", {})
            excl = full["wall_s"] - ph.get("load index", 0) - ph.get("device arena", 0) - ph.get("gpu runtime start", 0)
            body = open(sai, "rb").read()[64:]
            if base_sai is None:
                base_sai = body
            r = {"parse_only": po, "e2e": full, "reads_per_s_excl_load": n / excl,
                 "ingest_reads_per_s": n / max(po.get("parse_only", {}).get("wait_s", po["wall_s"]), 1e-9),
                 "sai_equal_plain": body == base_sai}
            res[name] = r
            log(f"{name}: e2e {r['reads_per_s_excl_load'] / 1e6:.2f} M reads/s excl. load, parse-only wait "
                f"{po.get('parse_only', {}).get('wait_s')} s, inflate {full.get('inflate')}, .sai equal {r['sai_equal_plain']}")
            os.unlink(sai)
            time.sleep(3.0)
    finally:
        subprocess.run(["rm", "-rf", d])
    line = json.dumps(res)
    print(line)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
