"""Host check of the round-1 size gates (hpc_suffix_array_amd/csrc/sa_limits.h):
g++ builds tests/cpp/limits_check.cpp, which finds the largest suffix count
whose per-XCD second-pass regions fit 32-bit offsets and checks the gate at
that boundary (past ~4.02e9 suffixes queue 7's offsets wrapped)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_xq_gate_at_the_32_bit_boundary(tmp_path):
    exe = tmp_path / "limits_check"
    subprocess.run(["g++", "-O2", "-std=c++17", os.path.join(ROOT, "tests", "cpp", "limits_check.cpp"), "-o",
                    str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "bad 0" in r.stdout
