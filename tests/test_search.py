"""The sampled lower bound of the sparse rank look-ups (interpolation-
guided search of the round-1 key samples, then a binary search over the
last 2^ksh slots; hpc_suffix_array_amd/csrc/sa_search.h) against
std::lower_bound on the host: g++ builds tests/cpp/search_check.cpp."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_lower_bound_sampled_matches_std(tmp_path):
    exe = tmp_path / "search_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "hpc_suffix_array_amd", "csrc"),
                    os.path.join(ROOT, "tests", "cpp", "search_check.cpp"), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.startswith("ok "), out.stdout
