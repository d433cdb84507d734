import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "my-lidar-graph-slam_amd")
for p in (PKG, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


@pytest.fixture(scope="session")
def world():
    from lgs_amd import scene
    return scene.make_world()


@pytest.fixture(scope="session")
def ctx():
    from lgs_amd import abi
    c = abi.Context(0)
    yield c
    c.close()


def launcher_cost(oracle=False):
    """CostGreedyEndpoint as CreateCostGreedyEndpoint builds it from the default
    JSON (C/slam_launcher.cpp:54-76): the (stddev, scale) arguments land in the
    (scale, stddev) slots, so mScalingFactor = 0.05 and mStandardDeviation = 1.0."""
    vals = (0.01, 20.0, 0.075, 0.1, 1, 0.05, 1.0)
    if oracle:
        import oracle_bind as ob
        return ob.CostGE(*vals)
    from lgs_amd import abi
    return abi.CostGEParams(*vals)
