timeout -k 10 300 python -u -m pytest tests/test_gpu_bb.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_bb.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_bb.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest.log 2>&1; tail -3 gpurun_out/pytest.log
