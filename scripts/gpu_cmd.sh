set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_random_configs.py -m gpu -q -rf --timeout 120 --timeout-method thread > gpurun_out/pytest_new.log 2>&1; rc=$?
tail -40 gpurun_out/pytest_new.log; exit $rc
