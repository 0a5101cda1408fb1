#!/bin/bash
# Round 5: config 2 with the periodic half-size resynthesis (k_fused MODE 4, pitch 2) vs the
# MODE 3 gather (PV_FUSED_HALF=0): fused + parity tests, then the c2 A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_parity.py tests/test_gpu_full_size.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ab/half_tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/ab/half_tests.log)"
[ $rc -ne 0 ] && { grep -E "assert|Error|FAILED" gpurun_out/ab/half_tests.log | head -12; exit $rc; }
AB_ARGS="--workload c2" AB_STEPS=400 bash scripts/ab.sh base:PV_FUSED_HALF=0 || exit $?
