# per-phase wall-clock probes of the batched pipeline (diagnostics build)
mkdir -p gpurun_out
LGS_LIB=my-lidar-graph-slam_amd/lgs_amd/liblgs_hip_probe.so timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --streams 1 --no-cpu --latency-calls 0 --loop-line 0 > gpurun_out/r02_probe.log 2>&1
