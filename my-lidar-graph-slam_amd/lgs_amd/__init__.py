"""Python plumbing around the MI355X hot-path library (liblgs_hip.so).

`abi`   ctypes binding of include/lgs_hip.h (the drop-in C-ABI)
`scene` synthetic worlds/scans for tests and bench.py

Import with the package directory on sys.path:
    sys.path.insert(0, "<repo>/my-lidar-graph-slam_amd"); import lgs_amd
"""
from . import abi, scene  # noqa: F401

__all__ = ["abi", "scene"]
