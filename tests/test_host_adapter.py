"""The NwAlignFn adapter file (gpuseqalign_amd/host/nwalign_amd.cpp)
compiles against the host mirror of the reference's types and behaves as an align slot must
without a device (tests/cpp/adapter_main.cpp); on the GPU its laps come through
gsa_set_lap_callback in the reference's order (test_gpu_laps.py)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST = os.path.join(ROOT, "gpuseqalign_amd", "host")
PKG = os.path.join(ROOT, "gpuseqalign_amd")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_adapter_compiles_and_runs_without_device(tmp_path):
    exe = str(tmp_path / "adapter_check")
    cmd = ["g++", "-O1", "-std=c++17", "-Wall", "-Wextra", "-Werror", "-I", HOST,
           os.path.join(ROOT, "tests", "cpp", "adapter_main.cpp"), os.path.join(HOST, "nwalign_amd.cpp"),
           os.path.join(HOST, "nw_host.cpp"), "-o", exe, "-L", PKG, "-lgsa", "-Wl,-rpath," + PKG]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60, env=dict(os.environ, HIP_VISIBLE_DEVICES=""))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "adapter check: ok" in r.stdout
