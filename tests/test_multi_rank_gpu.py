"""The N>1 path of bench.py on the GPU (configs[3]'s sharding, rehearsed on one MI355X):
torchrun starts 2 ranks before any GPU call; each builds its own index replica, aligns its own
read shard (shard_seed) through the HIP engine and dumps its hits.  The concatenation of the two
ranks' hits must equal a single process aligning both shards as one batch (--shards 2): sharding
by reads changes nothing in the results (the batch-level options of bwtaln.c:86-93 depend only
on the max read length, equal here)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--scale", "0.01", "--reads", "20000", "--steps", "1", "--warmup", "0", "--no-cpu", "--exact-leg", "0",
        "--sa2pos", "0"]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("aln", ["", "-n 0"])
def test_two_ranks_equal_one_batch(tmp_path, aln):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="4")
    d2 = str(tmp_path / "two")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
                        os.path.join(ROOT, "bench.py"), *ARGS, "--aln", aln, "--dump", d2],
                       capture_output=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    line = [x for x in r.stdout.decode().splitlines() if x.startswith("{")][-1]
    assert '"n_gpus": 2' in line
    d1 = str(tmp_path / "one")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *ARGS, "--aln", aln, "--shards", "2",
                        "--dump", d1], capture_output=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    a = [np.load(f"{d2}.rank{k}.npz") for k in (0, 1)]
    b = np.load(f"{d1}.rank0.npz")
    assert b["n_aln"].size == 40000 and all(x["n_aln"].size == 20000 for x in a)
    assert (np.concatenate([x["n_aln"] for x in a]) == b["n_aln"]).all()
    assert (np.concatenate([x["alns"] for x in a]) == b["alns"]).all()
    # with 1 % substitutions most 100 bp reads have no exact hit; the gapped search places most
    assert b["n_aln"].sum() > (10000 if aln else 30000)
