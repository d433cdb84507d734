set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_planes.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r02h_planes.log 2>&1
