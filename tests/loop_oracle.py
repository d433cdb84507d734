"""Oracle-side LoopDetectorRealTimeCorrelative::Detect producing the same
176-byte records as lgs_loop_detect_rtcsm (test infrastructure only)."""
import ctypes as C

import numpy as np

import oracle_bind as ob
from lgs_amd import abi
from lgs_amd.loopbatch import RECORD_BYTES


def oracle_detect_fn(maps, cands, params, cost, thr):
    """params/cost: tuples in lgs_rtcsm_params / lgs_cost_ge_params order."""
    grids = {}

    def fn(subq, lo, hi):
        out = np.zeros((hi - lo, RECORD_BYTES), dtype=np.uint8)
        for q, first, count in subq:
            if q not in grids:
                m = maps[q]
                coarse = ob.precompute(m.cells, params[0])
                grids[q] = (ob.OGrid(m.cells, m.min_x, m.min_y, m.res), ob.OGrid(coarse, m.min_x, m.min_y, m.res))
            g, cg = grids[q]
            m = maps[q]
            for j in range(first, first + count):
                c = cands[lo + j]
                s = ob.Summary()
                ob.lib().orc_rtcsm_optimize_pose(C.byref(g.g), C.byref(cg.g), C.byref(ob.RtcsmParams(*params)),
                                                 C.byref(ob.CostGE(*cost)), C.byref(ob.OScan(c.ranges, c.angles).s),
                                                 ob.Pose(*c.pose), thr, C.byref(s))
                r = abi.LoopResult()
                r.found = s.pose_found
                r.start_node_index = m.node_index
                r.end_node_index = c.node_index
                r.start_node_pose = abi.Pose2D(*m.node_pose)
                e = s.estimated_pose
                r.estimated_pose = abi.Pose2D(e.x, e.y, e.theta)
                if s.pose_found:
                    rel = ob.lib().orc_inverse_compound(ob.Pose(*m.node_pose), e)
                    r.relative_pose = abi.Pose2D(rel.x, rel.y, rel.theta)
                for k in range(9):
                    r.covariance[k] = s.covariance[k]
                r.score = s.score_max
                r.normalized_cost = s.normalized_cost
                out[j] = np.frombuffer(bytes(r), dtype=np.uint8)
        return out

    return fn
