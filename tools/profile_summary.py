#!/usr/bin/env python3
"""Summarise a tools/profile_round.sh directory into profiles/<round>_<tag>_*.

kernel_stats.csv: the rocprofv3 --stats table of the kernel-trace pass (copied).
pmc.json: per kernel of the hot path -- dispatches, average duration (trace pass),
and per-dispatch L2<->fabric request counts with the bytes they imply:
  read bytes  = 128 x RDREQ_128B + 64 x RDREQ_64B + 32 x RDREQ_32B
  write bytes = 64 x WRREQ_64B + 32 x (WRREQ - WRREQ_64B)
(MI355X_MICROARCH.md, HBM section: the EA counters see every L2 miss that leaves
the XCD, Infinity-Cache hits included; RDREQ_DRAM is the share sent to DRAM).
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

HOT = ("k_exact", "k_pack_reads", "k_gapped", "k_width", "k_search", "k_sw", "k_coop_roots", "k_coop", "k_sa2pos", "k_expand_sa")


def short(name):
    for h in HOT:
        if h in name:
            return h + ("<wide>" if "k_gapped" in name and "ILb1E" in name else "")
    return None


def main():
    out, rnd, tag = sys.argv[1], sys.argv[2], sys.argv[3]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prof = os.path.join(root, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = glob.glob(f"{out}/trace/**/run_kernel_stats.csv", recursive=True)
    if stats:
        shutil.copy(stats[0], os.path.join(prof, f"{rnd}_{tag}_kernel_stats.csv"))
    # durations per kernel from the trace pass
    dur = defaultdict(list)
    for f in glob.glob(f"{out}/trace/**/run_kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if k:
                dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    # counters per kernel per dispatch
    cnt = defaultdict(lambda: defaultdict(float))
    ndisp = defaultdict(set)
    for f in glob.glob(f"{out}/pmc*/**/run_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if k:
                cnt[k][r["Counter_Name"]] += float(r["Counter_Value"])
                ndisp[k].add((f, r["Dispatch_Id"]))
    res = {"round": rnd, "tag": tag, "kernels": {}}
    for log in [f"{out}/trace.json"]:
        try:
            res["bench_line"] = json.loads(open(log).read().strip().splitlines()[-1])
        except Exception:
            pass
    line = res.get("bench_line", {})
    main_exact = "-n 0" in str(line.get("config", {}).get("aln_options", ""))
    leg = line.get("extra", {}).get("exact_leg") or {}
    res["workloads"] = [w for w in (line.get("config", {}).get("workload"), leg.get("workload")) if w]

    def runs_of(k):
        """aln runs (ibwa_batch_run calls) of the profiled command in which kernel k ran."""
        main = line.get("steps", 0) + line.get("warmup", 0)
        if k in ("k_exact", "k_pack_reads") and not main_exact:
            return leg.get("steps", 0) + 1 if leg else 0
        return main
    for k in sorted(set(dur) | set(cnt)):
        c = cnt.get(k, {})
        # each pmc pass ran the same dispatches: per-dispatch = sum / dispatches of that pass
        n_pass = max(1, len({d for d in ndisp[k] if "pmc1" in d[0]}))
        g = lambda n: c.get(n, 0.0) / n_pass
        rd = 128 * g("TCC_EA0_RDREQ_128B_sum") + 64 * g("TCC_EA0_RDREQ_64B_sum") + 32 * g("TCC_EA0_RDREQ_32B_sum")
        wr = 64 * g("TCC_EA0_WRREQ_64B_sum") + 32 * (g("TCC_EA0_WRREQ_sum") - g("TCC_EA0_WRREQ_64B_sum"))
        d = dur.get(k, [])
        res["kernels"][k] = {
            "dispatches_traced": len(d), "avg_ms": sum(d) / len(d) if d else None,
            "per_dispatch": {n.replace("_sum", ""): g(n) for n in sorted(c)},
            "read_bytes_per_dispatch": rd, "write_bytes_per_dispatch": wr,
            "dram_read_fraction": (g("TCC_EA0_RDREQ_DRAM_sum") / g("TCC_EA0_RDREQ_sum")) if g("TCC_EA0_RDREQ_sum") else None,
            # over all dispatches of the command (a step runs several launches of some kernels)
            "total_ms": sum(d), "total_read_bytes": rd * n_pass, "total_write_bytes": wr * n_pass,
            "runs": runs_of(k),
        }
    path = os.path.join(prof, f"{rnd}_{tag}_pmc.json")
    json.dump(res, open(path, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
