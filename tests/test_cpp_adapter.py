"""The reference-shaped C++ adapter (my-lidar-graph-slam_amd/host/) through its
C++ test driver (tests/cpp/adapter_test.cpp, built by `make cpptest`)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "build", "adapter_test")


def run():
    assert os.path.exists(BIN), "build first: make -C <repo> all"
    return subprocess.run([BIN], capture_output=True, text=True, timeout=600)


def test_adapter_links_and_reports_missing_device():
    """CPU: the adapter, the C-ABI library and the oracle load; without a GPU
    the driver exits with the skip status after Device() threw lgs::hip::Error
    (with one, it runs the GPU checks and must pass them)."""
    r = run()
    if r.returncode == 0 and "ADAPTER TESTS PASSED" in r.stdout:
        pytest.skip("a GPU is present: covered by the gpu test")
    assert r.returncode == 77, r.stdout + r.stderr
    assert "no GPU" in r.stdout


@pytest.mark.gpu
def test_adapter_on_gpu():
    r = run()
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ADAPTER TESTS PASSED" in r.stdout
