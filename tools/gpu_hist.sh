set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_cpp_adapter.py tests/test_gpu_batch.py -m gpu -x -q -s --timeout 120 --timeout-method thread > gpurun_out/r02c_hist.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py -m gpu -x -q -s --timeout 120 --timeout-method thread > gpurun_out/r02c_hist2.log 2>&1
true
