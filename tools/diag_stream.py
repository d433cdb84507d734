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
odo = len(sys.argv) > 2 and sys.argv[2] == "odo"   # odometry guesses (bench.py run_stream) instead of the truth
ctx = abi.Context(0)
world = scene.make_world()
ang = scene.beam_angles(1081)
n = int(os.environ.get('DIAG_STEPS', 40))
slow_ms = float(os.environ.get('DIAG_SLOW_MS', 0))
truths = [(5.0 * np.cos(0.02 * k), 5.0 * np.sin(0.02 * k), 0.02 * k + np.pi / 2) for k in range(n)]
bp = abi.BuilderParams(0.01, 20.0, 0.6, 0.45)
P, cost = abi.RtcsmParams(5, *win, 20.0), abi.CostGEParams(0.01, 20.0, 0.075, 0.1, 1, 0.05, 1.0)
latest = ctx.map(0.05, 100, 200, 200, center=truths[0][:2])
scans = [ctx.interpolate(ctx.scan(scene.ray_cast(world, t, ang), ang), 0.05, 0.25) for t in truths]
ctx.set_option(abi.LGS_OPT_PROFILE, 1)
ctx.set_option(abi.LGS_OPT_PROFILE_MASK, (1 << len(abi.KERNEL_IDS)) - 1)
rng = np.random.default_rng(7)
est = [truths[0]]


def odometry(last):
    d = (0.1 + rng.normal(0, 0.01), rng.normal(0, 0.01), 0.02 + rng.normal(0, 0.005))
    c, s = np.cos(last[2]), np.sin(last[2])
    return (last[0] + c * d[0] - s * d[1], last[1] + s * d[0] + c * d[1], last[2] + d[2])


for k in range(1, n):
    lo = max(0, k - 10)
    poses = est if odo else truths
    guess = odometry(est[-1]) if odo else truths[k]
    latest.construct(scans[lo:k], poses[lo:k], bp)
    g = latest.geometry()
    ctx.reset_stats()
    t0 = time.perf_counter()
    out = ctx.optimize_pose_query(latest.grid(), P, cost, scans[k], guess)
    e = out.estimated_pose
    est.append((e.x, e.y, e.theta))
    dt = 1e3 * (time.perf_counter() - t0)
    st = ctx.kernel_stats()
    ks = " ".join(f"{name}={v['total_ms']:.3f}" for name, v in st.items() if v["launches"])
    if dt < slow_ms:
        continue
    print(f"k={k} map={g['w']}x{g['h']} {dt:.3f} ms coarse={out.coarse_blocks} fine={out.fine_blocks} "
          f"slow={out.slow_path} guard={out.guard_hits} fix={out.fixups} win={list(out.win)} best={list(out.best_win)} score={out.score_max:.4f} | {ks}", flush=True)
