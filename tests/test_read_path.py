"""samse/sampe's read path (sam_common.h take_reads: the bulk FASTQ parser's records converted by
rec_to_read on host threads, the serial reader taking over at the first record the bulk parser does
not take) against next_read alone (bwa_read_seq, bwaseqio.c:145-208) as whole Read objects -- name,
codes, quality, reverse complement, lengths, barcode -- with a barcode (-B), Illumina 1.3 qualities
(-I) and quality trimming (-q) in the mode, in batches whose buffers are reused like sampe's.  CPU
only: builds tools/read_check.cpp with g++ (the GPU tests run the same path through the CLI)."""
import os
import subprocess
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from test_fastq_bulk import CASES  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MODES = {"plain": (0x02, 0), "barcode5": (0x02 | 5 << 24, 0), "il13_q15": (0x202, 15), "q20": (0x02, 20)}


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("rc") / "read_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", "-I", os.path.join(ROOT, "ibwa_amd", "csrc"),
                    "-I", os.path.join(ROOT, "include"), "-o", exe, os.path.join(ROOT, "tools", "read_check.cpp"), "-lz"],
                   check=True)
    return exe


@pytest.mark.parametrize("name", sorted(CASES))
@pytest.mark.parametrize("mode", sorted(MODES))
def test_batches_equal_serial_reads(checker, tmp_path, name, mode):
    p = tmp_path / f"{name}.fq"
    p.write_bytes(CASES[name]().encode())
    m, q = MODES[mode]
    for batch, threads in ((1000, 4), (7, 3)):
        r = subprocess.run([checker, str(p), hex(m), str(q), str(batch), str(threads)], capture_output=True, text=True)
        assert r.returncode == 0 and r.stdout.startswith("OK"), (name, mode, batch, r.stdout[-2000:], r.stderr[-500:])
