"""The multi-rank loop-closure path run by real processes on the GPU
(loop_detector_real_time_correlative.cpp:38-93).

One GPU box has one device, so these tests put two ranks on device 0 and
gather over gloo (RCCL refuses two ranks on one device); what they exercise is
everything a rank of an 8-GPU run does besides the xGMI transfer: its own
process and HIP context, loopbatch.run_sharded with the HIP matcher
(hip_detect_fn) on its contiguous candidate block, the all-gather of the
176-byte records and the reorder.  The gathered records must be byte-identical
to one process matching every candidate.  No scaling number comes from here
(DESIGN §7): ranks sharing one GPU share its CUs.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import test_loopbatch_cpu as small
from lgs_amd import abi, loopbatch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    """One rank: its own process and HIP context on device 0, gloo group."""
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ctx = abi.Context(0)
    maps, cands = small.make_problem()
    fn = loopbatch.hip_detect_fn(ctx, maps, cands, abi.RtcsmParams(*small.PARAMS), abi.CostGEParams(*small.COST),
                                 small.THR)
    for rep in range(2):   # twice: the second call reuses the rank's uploaded maps and scans
        rec = loopbatch.run_sharded(cands, fn, rank, world, dist)
        np.save(os.path.join(out, f"r{rank}_{rep}.npy"), rec)
    dist.barrier()
    dist.destroy_process_group()
    ctx.close()


def _spawn(world, out):
    port = _free_port()
    env = dict(os.environ, PYTHONPATH=os.pathsep.join(
        [os.path.join(ROOT, "my-lidar-graph-slam_amd"), os.path.join(ROOT, "tests"), os.environ.get("PYTHONPATH", "")]))
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "worker", str(r), str(world), str(port),
                               str(out)], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
             for r in range(world)]
    logs = []
    for p in procs:
        try:
            o, _ = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        logs.append((p.returncode, o))
    return logs


@pytest.mark.parametrize("world", [2, 3])
def test_ranks_as_processes_gather_identical_records(ctx, tmp_path, world):
    maps, cands = small.make_problem()
    p, c = abi.RtcsmParams(*small.PARAMS), abi.CostGEParams(*small.COST)
    single = loopbatch.run_sharded(cands, loopbatch.hip_detect_fn(ctx, maps, cands, p, c, small.THR))
    for rc, log in _spawn(world, tmp_path):
        assert rc == 0, log[-3000:]
    for r in range(world):
        for rep in range(2):
            got = np.load(tmp_path / f"r{r}_{rep}.npy")
            assert got.tobytes() == single.tobytes(), (r, rep)
    found = loopbatch.loop_results(single)
    assert 0 < len(found) < len(cands)


def test_bench_loop_line_two_ranks_rehearsal():
    """bench.py --gpus 2 itself (torchrun child, two ranks, LGS_BENCH_REHEARSE:
    both on device 0, gloo): the loop line's ranks shard the 512 candidates
    and gather them; the found count equals the one-rank run's."""
    lines = {}
    for world in (1, 2):
        env = dict(os.environ, LGS_BENCH_REHEARSE="1")
        r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--workload", "loop",
                            "--steps", "2", "--warmup", "1", "--no-cpu"], cwd=ROOT, env=env, capture_output=True,
                           text=True, timeout=400)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
        lines[world] = json.loads(r.stdout.strip().splitlines()[-1])
    assert lines[2]["n_gpus"] == 2 and lines[1]["n_gpus"] == 1
    assert lines[2]["config"]["candidates"] == lines[1]["config"]["candidates"] == 512
    assert lines[2]["config"]["found"] == lines[1]["config"]["found"] > 0


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "worker":
    _worker(int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5])
