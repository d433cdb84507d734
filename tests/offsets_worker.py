"""Worker of tests/test_gpu_offsets.py, run in its own process with LGS_LIB =
liblgs_hip_checked.so (the checked build: every coarse / superblock plane
offset a correlative consumer forms or reads is tested against its padded
plane, LGS_CHECK_OFFSETS).  Runs bench.py's config-2 workload through every
row contract -- lean rows (default), materialised rows, poisoned workspaces,
forced guard fix-ups, a lone call, the dense path, loop-detector windows --
and writes the checks' counters and the lean batch's records as JSON.
Usage: offsets_worker.py OUT.json"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "my-lidar-graph-slam_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

import bench  # noqa: E402
from conftest import launcher_cost  # noqa: E402
from lgs_amd import abi, scene  # noqa: E402


def _record(out):
    return [bool(out.pose_found), list(out.best_win), out.score_max, list(out.estimated_pose.tuple()),
            out.normalized_cost, out.coarse_blocks, out.fine_blocks]


def main(path):
    assert os.environ.get("LGS_LIB", "").endswith("liblgs_hip_checked.so"), os.environ.get("LGS_LIB")
    ctx = abi.Context(0)
    world = scene.make_world()
    ang = scene.beam_angles(1081)
    cells, mx, my = bench.bench_map(world, ang)
    scans, inits, _ = bench.random_scans(world, ang, np.random.default_rng(1000), 64)
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    ds = [ctx.scan(r, ang) for r in scans]
    cost = launcher_cost()
    P = abi.RtcsmParams(*bench.PARAMS)
    ctx.offset_checks(reset=True)
    runs, records = {}, None

    def run(name, opts, fn):
        for k, v in opts:
            ctx.set_option(k, v)
        try:
            res = fn()
        finally:
            for k, v in opts:
                ctx.set_option(k, {abi.LGS_OPT_LEAN_PROJECT: 1, abi.LGS_OPT_GUARD_EPS: 1e-9}.get(k, 0))
        runs[name] = ctx.offset_checks(reset=True)
        return res

    records = [_record(o) for o in run("lean", [], lambda: ctx.optimize_pose_query_batch(g, P, cost, ds, inits))]
    run("materialised", [(abi.LGS_OPT_LEAN_PROJECT, 0)],
        lambda: ctx.optimize_pose_query_batch(g, P, cost, ds[:32], inits[:32]))
    run("lean_poisoned", [(abi.LGS_OPT_POISON_WS, 1)],
        lambda: ctx.optimize_pose_query_batch(g, P, cost, ds[:32], inits[:32]))
    run("materialised_poisoned", [(abi.LGS_OPT_LEAN_PROJECT, 0), (abi.LGS_OPT_POISON_WS, 1)],
        lambda: ctx.optimize_pose_query_batch(g, P, cost, ds[32:48], inits[32:48]))
    run("guard_fixups", [(abi.LGS_OPT_INJECT_INDEX, 1), (abi.LGS_OPT_GUARD_EPS, 1e-5)],
        lambda: ctx.optimize_pose_query_batch(g, P, cost, ds[48:64], inits[48:64]))
    run("lone", [], lambda: ctx.optimize_pose_query(g, P, cost, ds[0], inits[0]))
    run("dense", [(abi.LGS_OPT_FORCE_DENSE, 1)], lambda: ctx.optimize_pose_query(g, P, cost, ds[1], inits[1]))
    PL = abi.RtcsmParams(*bench.LOOP_PARAMS)
    run("loop_window", [], lambda: ctx.optimize_pose_query_batch(g, PL, cost, ds[:16], inits[:16]))
    with open(path, "w") as f:
        json.dump(dict(runs=runs, records=records), f)
    ctx.close()


if __name__ == "__main__":
    main(sys.argv[1])
