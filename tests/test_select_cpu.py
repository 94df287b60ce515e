"""CPU check of csrc/skm_select.h -- the device's restatement of GNU libstdc++ std::nth_element
and of the older Boost.Math median / median_absolute_deviation sequence (mad_mode 1,
call_functions.tcc:51-53) -- against std::nth_element itself (tests/native/select_check.cpp,
compiled here with g++): identical permutations and identical (median, MAD) bits on 20,000
tie-heavy, presorted and reversed arrays of up to 20,000 values."""
import os
import subprocess

from conftest import ROOT


def test_nth_element_restatement_matches_libstdcxx(tmp_path):
    exe = str(tmp_path / "select_check")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "signature_kmers_amd", "csrc"),
                           os.path.join(ROOT, "tests", "native", "select_check.cpp"), "-o", exe])
    p = subprocess.run([exe, "20000"], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "bad_perm 0 bad_stat 0" in p.stdout


def test_host_pool_runs_every_part_once(tmp_path):
    """csrc/skm_pool.h (skm_build_add_batch's packing threads): every part of 2,000 back-to-back runs
    of 0..299 parts executes exactly once on 1 / 2 / 7 / 16 threads, and the byte-balanced parallel
    packing of 20,000 random sequences equals the serial one (tests/native/pool_check.cpp)."""
    exe = str(tmp_path / "pool_check")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-pthread", "-I",
                           os.path.join(ROOT, "signature_kmers_amd", "csrc"),
                           os.path.join(ROOT, "tests", "native", "pool_check.cpp"), "-o", exe])
    p = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0 and "pool bad 0" in p.stdout, p.stdout + p.stderr
