"""Checked build: the correlative
consumers of bench.py's config-2 workload, run from liblgs_hip_checked.so
(LGS_CHECK_OFFSETS), test every coarse / superblock plane offset they form
(lean rows) or read (materialised rows) against its padded plane.  Over lean,
materialised and poisoned workspaces, forced guard fix-ups, a lone call, the
dense path and loop-detector windows: offsets were checked, none fell outside
its plane, and the checked build's records equal the product build's.

The checked library runs in a child process (the product library is the one
this process has loaded)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import launcher_cost
from lgs_amd import abi

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
CHECKED = os.path.join(os.path.dirname(abi.LIB_PATH), "liblgs_hip_checked.so")


def test_plane_offsets_inside_their_planes(ctx, tmp_path):
    from lgs_amd import scene
    from test_gpu_benchcfg import _bench
    from offsets_worker import _record

    assert os.path.exists(CHECKED), f"checked build missing: {CHECKED} (make -C my-lidar-graph-slam_amd/csrc)"
    out = tmp_path / "offsets.json"
    env = dict(os.environ, LGS_LIB=CHECKED)
    r = subprocess.run([sys.executable, "-u", os.path.join(HERE, "offsets_worker.py"), str(out)], env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    res = json.loads(out.read_text())
    for name, c in res["runs"].items():
        assert c["violations"] == 0, (name, c, hex(c["first"]))
    # every row contract was exercised (the small loop window may take
    # another path; the others stage or form rows)
    for name in ("lean", "materialised", "lean_poisoned", "materialised_poisoned", "guard_fixups", "lone", "dense"):
        assert res["runs"][name]["checked"] > 0, (name, res["runs"][name])
    # the product build's records for the same batch
    bench = _bench()
    world = scene.make_world()
    ang = scene.beam_angles(1081)
    cells, mx, my = bench.bench_map(world, ang)
    scans, inits, _ = bench.random_scans(world, ang, np.random.default_rng(1000), 64)
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    ds = [ctx.scan(rr, ang) for rr in scans]
    outs = ctx.optimize_pose_query_batch(g, abi.RtcsmParams(*bench.PARAMS), launcher_cost(), ds, inits)
    prod = json.loads(json.dumps([_record(o) for o in outs]))
    assert prod == res["records"]
