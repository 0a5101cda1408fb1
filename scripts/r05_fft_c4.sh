#!/bin/bash
# Round 5: FFT op (n = 2048 two-wave kernel) tests + fft_bench, and the config-4 run-length sweep.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fft.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_fft_tests.log 2>&1 || { tail -30 gpurun_out/r05_fft_tests.log; exit 1; }
tail -1 gpurun_out/r05_fft_tests.log
timeout -k 10 200 ./phase-vocoder_amd/build/fft_bench bench > gpurun_out/r05_fft_bench.jsonl 2>&1 || { cat gpurun_out/r05_fft_bench.jsonl; exit 1; }
cat gpurun_out/r05_fft_bench.jsonl
AB_VAR=PV_RUN_FRAMES AB_VALS="${C4_F:-16 24 32}" AB_WL=c4 bash scripts/ab_env.sh
