#!/bin/bash
# Round 5: balanced single launch (config 2): fused tests, A/B against uniform runs, stamps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_fused_bal_tests.log 2>&1 || { tail -30 gpurun_out/r05_fused_bal_tests.log; exit 1; }
tail -1 gpurun_out/r05_fused_bal_tests.log
AB_VAR=PV_FUSED_BALANCE AB_VALS="0 1" AB_WL=c2 AB_ARGS="--steps 400" bash scripts/ab_env.sh || exit 1
for b in 1 0; do
  PV_FUSED_BALANCE=$b PV_LIB_PATH=$PWD/phase-vocoder_amd/build/variants/libpv_stamps.so timeout -k 10 120 python scripts/fused_stamps.py > gpurun_out/r05_stamps_bal$b.json || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/r05_stamps_bal$b.json')); print('bal$b', d['launch_span_us'], d['waves'], d['placement'], d['frame_us'], d['setup_us'], d['seams_us'])"
done
