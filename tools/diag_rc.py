import sys, numpy as np
sys.path.insert(0,'my-lidar-graph-slam_amd'); sys.path.insert(0,'tests')
import oracle_bind as ob
from lgs_amd import abi, scene
ctx = abi.Context(0)
world = scene.make_world()
ang = scene.beam_angles(1081)
BP=(0.01,20.0,0.6,0.45)
gm = ctx.map(0.05, 100, 1000, 1000); om = ob.OMap(0.05, 100, 1000, 1000)
for k, p in enumerate(scene.arc_poses(10)):
    r = scene.ray_cast(world, p, ang)
    gm.update_scan(ctx.scan(r, ang), p, abi.BuilderParams(*BP)); om.integrate(p, ob.OScan(r, ang), ob.BuilderParams(*BP))
    c, h, m = gm.download()
    oc, oh, omm = om.cells(), om.hits(), om.misses()
    print(k, 'hits sum', h.sum(), oh.sum(), 'miss sum', m.sum(), omm.sum())
    d = np.argwhere(h != oh); print('hit diffs', len(d), d[:5].tolist(), [ (int(h[tuple(x)]), int(oh[tuple(x)])) for x in d[:5]])
    d = np.argwhere(m != omm); print('miss diffs', len(d), d[:5].tolist(), [ (int(m[tuple(x)]), int(omm[tuple(x)])) for x in d[:5]])
    d = np.argwhere(c != oc); print('cell diffs', len(d))
