"""The host copy pool (csrc/copy_pool.cpp) on the CPU: its streaming gather
of strided rows into contiguous destinations, the tee to a second
destination and zero fills, against plain copies (tests/native/
copy_pool_check.cpp, compiled here with g++)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd", "csrc")


def test_copy_pool_gathers_and_tees(tmp_path):
    exe = str(tmp_path / "copy_pool_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-DRSAMD_TUNING_ENV=0", "-I", CSRC,
                    os.path.join(ROOT, "tests", "native", "copy_pool_check.cpp"),
                    os.path.join(CSRC, "copy_pool.cpp"), "-pthread", "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:]
    assert "0 bad" in r.stdout
