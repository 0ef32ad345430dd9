"""The kernels' division by invariant integers (raytracert_amd/csrc/fastdiv.h, used to decode
sample and tile indices): the same header built for the host by g++ equals '/' and '%' on every
divisor up to 4096 and sampled larger ones, edge and random numerators."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_fastdiv_matches_integer_division(tmp_path):
    exe = str(tmp_path / "fastdiv_check")
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-Werror", "-I" + os.path.join(ROOT, "raytracert_amd", "csrc"),
                    os.path.join(ROOT, "tests", "cxx", "fastdiv_check.cpp"), "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.startswith("ok "), r.stdout
