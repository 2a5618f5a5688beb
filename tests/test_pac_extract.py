"""The .pac extraction samse/sampe use for MD/NM, refinement and mate-rescue windows (sam_common.h
extract, dbset_extract_sequence dbset.c:306-325): four codes per byte against bns_pac base by base,
for one reference and for several read back to back, at random starts and lengths, ranges past the
end included.  CPU only: builds tools/pac_check.cpp with g++."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("pac") / "pac_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", "-I", os.path.join(ROOT, "ibwa_amd", "csrc"),
                    "-I", os.path.join(ROOT, "include"), "-o", exe, os.path.join(ROOT, "tools", "pac_check.cpp"), "-lz"],
                   check=True)
    return exe


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_unpacked_windows_equal_base_by_base(checker, seed):
    r = subprocess.run([checker, str(seed)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "OK", r.stdout


@pytest.fixture(scope="module")
def md_checker(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("md") / "md_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", "-I", os.path.join(ROOT, "ibwa_amd", "csrc"),
                    "-I", os.path.join(ROOT, "include"), "-o", exe, os.path.join(ROOT, "tools", "md_check.cpp"), "-lz"],
                   check=True)
    return exe


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_md_equals_base_by_base(md_checker, seed):
    """cal_md1 (MD / NM of samse and sampe, eight bases compared at a time) against bwa_cal_md1 base by
    base: reads with substitutions and N's, with and without CIGARs, windows past the reference's end."""
    r = subprocess.run([md_checker, str(seed)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "OK", r.stdout
