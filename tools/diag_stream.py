"""Diagnostics: per-step match details of the config-4 frontend with the
config-2 window (why is a lone match against the latest map slow?)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "my-lidar-graph-slam_amd"))
from lgs_amd import abi, scene  # noqa: E402

win = (4.0, 4.0, 1.0471976) if len(sys.argv) < 2 else tuple(float(v) for v in sys.argv[1].split(","))
ctx = abi.Context(0)
world = scene.make_world()
ang = scene.beam_angles(1081)
n = 40
truths = [(5.0 * np.cos(0.02 * k), 5.0 * np.sin(0.02 * k), 0.02 * k + np.pi / 2) for k in range(n)]
bp = abi.BuilderParams(0.01, 20.0, 0.6, 0.45)
P, cost = abi.RtcsmParams(5, *win, 20.0), abi.CostGEParams(0.01, 20.0, 0.075, 0.1, 1, 0.05, 1.0)
latest = ctx.map(0.05, 100, 200, 200, center=truths[0][:2])
scans = [ctx.interpolate(ctx.scan(scene.ray_cast(world, t, ang), ang), 0.05, 0.25) for t in truths]
ctx.set_option(abi.LGS_OPT_PROFILE, 1)
ctx.set_option(abi.LGS_OPT_PROFILE_MASK, (1 << len(abi.KERNEL_IDS)) - 1)
for k in range(1, n):
    lo = max(0, k - 10)
    latest.construct(scans[lo:k], truths[lo:k], bp)
    g = latest.geometry()
    ctx.reset_stats()
    t0 = time.perf_counter()
    out = ctx.optimize_pose_query(latest.grid(), P, cost, scans[k], truths[k])
    dt = 1e3 * (time.perf_counter() - t0)
    st = ctx.kernel_stats()
    ks = " ".join(f"{name}={v['total_ms']:.3f}" for name, v in st.items() if v["launches"])
    print(f"k={k} map={g['w']}x{g['h']} {dt:.3f} ms coarse={out.coarse_blocks} fine={out.fine_blocks} "
          f"slow={out.slow_path} guard={out.guard_hits} fix={out.fixups} win={list(out.win)} | {ks}", flush=True)
