timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest.log 2>&1; tail -2 gpurun_out/pytest.log
for q in 1 0; do :; done; for q in 1 0; do
  timeout -k 10 300 python bench.py --no-cpu --steps 40 --warmup 5 --latency-calls 30 --super-quad $q > gpurun_out/ab_q$q.log 2>&1 || exit $?
done
echo done
