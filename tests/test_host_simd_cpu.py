"""csrc/host_simd.cpp's cell conversion (the latest-map step's hit points ->
cells, WorldCoordinateToGridCellIndex H/grid_map/grid_map.hpp:779-790) is
exactly floor((x - min) / res): built and run on the host."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "..", "my-lidar-graph-slam_amd", "csrc", "host_simd.cpp")


def test_cells_of_points_exact(tmp_path):
    exe = tmp_path / "host_simd_check"
    subprocess.run(["g++", "-O3", "-std=c++17", "-ffp-contract=off", os.path.join(HERE, "cpp", "host_simd_check.cpp"),
                    SRC, "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches 0" in r.stdout
