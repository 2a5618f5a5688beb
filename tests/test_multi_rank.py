"""The N>1 path of bench.py on CPU (gloo, world size 2).

Reads shard with no exchange step: each rank aligns its own disjoint reads
(`bench.shard_seed`) against a full index replica and the only collective is
the max over ranks of the timed region (`bench.reduce_max`).  Checked here:
shards are disjoint and deterministic, the per-rank results concatenated equal
one process aligning all shards (reads are independent; fixed read length keeps
the batch-level options equal), and the max-reduce returns the slowest rank.
The alignment itself is the CPU restatement (this container has no GPU).
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import bench
import oracle
from tests.synth_util import golden_genome_ascii, synth_reads

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
N_PER_RANK = 300


def _encode(reads):
    recs = [(f"r{i}", s.encode(), b"I" * len(s)) for i, s in enumerate(reads)]
    opt = oracle.default_opt()
    return oracle.encode_reads(recs, opt.mode, 0)


def _shard(rank):
    genome, _, lens = golden_genome_ascii()
    return synth_reads(genome, lens, bench.shard_seed(rank), N_PER_RANK, 100, 0.01, 0.05)


def _align(reads):
    b0 = oracle.Bwt(os.path.join(GOLD, "g1m.bwt"))
    b1 = oracle.Bwt(os.path.join(GOLD, "g1m.rbwt"))
    seq, off, lns = _encode(reads)
    n_aln, alns, _ = oracle.cal_sa_reg_gap(b0, b1, seq, off, lns, oracle.default_opt(), n_threads=2)
    return n_aln, alns


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        reads = _shard(rank)
        n_aln, alns = _align(reads)
        # the slowest rank's time is what the job reports
        t = bench.reduce_max(1.0 + rank, dist, "cpu")
        got = [None] * world
        dist.all_gather_object(got, (reads, n_aln.tolist(), alns.tobytes()))
        if rank == 0:
            q.put((t, got))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_ranks_shard_and_reduce():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    t, got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert t == 2.0
    shards = [g[0] for g in got]
    assert set(shards[0]).isdisjoint(shards[1])
    assert shards[0] == _shard(0) and shards[1] == _shard(1)
    n_all, a_all = _align(shards[0] + shards[1])
    assert np.concatenate([np.array(g[1], np.int32) for g in got]).tolist() == n_all.tolist()
    assert b"".join(g[2] for g in got) == a_all.tobytes()


def test_reduce_max_single_process():
    assert bench.reduce_max(3.5, None, "cpu") == 3.5


@pytest.mark.parametrize("rank", [0, 1, 7])
def test_shard_seeds_distinct(rank):
    assert bench.shard_seed(rank) != bench.shard_seed(rank + 1)
