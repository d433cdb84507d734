for bs in 64:1 128:1 64:2 128:2; do
  b=${bs%%:*}; s=${bs##*:}
  timeout -k 10 300 python bench.py --no-cpu --steps 40 --warmup 3 --latency-calls 0 --batch $b --streams $s > gpurun_out/ab_b${b}_s${s}.log 2>&1 || exit $?
done
echo done
