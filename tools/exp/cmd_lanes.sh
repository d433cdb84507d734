timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest.log 2>&1; tail -2 gpurun_out/pytest.log
for m in 2 100 1; do
  timeout -k 10 300 python bench.py --no-cpu --steps 40 --warmup 5 --latency-calls 50 --lanes-min-batch $m > gpurun_out/ab_lmb$m.log 2>&1 || exit $?
done
echo done
