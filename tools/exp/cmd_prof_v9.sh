#!/bin/bash
# r01 v9 evidence: kernel trace + PMC passes of the default command, every bench line, K3 rebuild trace
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS=200 WARMUP=10 bash tools/gpu_prof.sh r01v9 || exit $?
echo "== bench default"
timeout -k 10 300 python bench.py > gpurun_out/bench_match.json 2> gpurun_out/bench_match.err || exit $?
cat gpurun_out/bench_match.json
WORKLOADS="refine loop loop_bb stream rebuild" bash tools/gpu_bench_all.sh || exit $?
echo "== rebuild trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_rebuild_r01v9 -o run -- \
  python3 bench.py --workload rebuild --no-cpu --steps 20 > gpurun_out/trace_rebuild_r01v9.log 2>&1 || exit $?
echo done
