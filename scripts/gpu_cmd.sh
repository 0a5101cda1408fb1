set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -rf --timeout 120 --timeout-method thread -k "capacity or two_handles" > gpurun_out/pytest_new.log 2>&1; rc=$?
tail -30 gpurun_out/pytest_new.log; exit $rc
