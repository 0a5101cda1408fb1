#!/bin/bash
# Round 5: FFT op n = 32 / 64 on T = n/8 lanes per transform (k_fft_t8): tests + fft_bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fft.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_fft_small_tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/r05_fft_small_tests.log)"
[ $rc -ne 0 ] && { grep -E "assert|Error|FAILED" gpurun_out/r05_fft_small_tests.log | head -12; exit $rc; }
timeout -k 10 200 ./phase-vocoder_amd/build/fft_bench bench > gpurun_out/r05_fft_bench2.jsonl 2>&1 || { cat gpurun_out/r05_fft_bench2.jsonl; exit 1; }
cat gpurun_out/r05_fft_bench2.jsonl
