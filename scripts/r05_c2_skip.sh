#!/bin/bash
# Round 5: config-2 single launch without the unread bins' analysis (pitch 2.0: bins > 256),
# and k_fused compiled for 3 waves/SIMD (the balanced launch holds 3 workgroups per CU):
# fused tests on base and fw3, then the c2 A/B base / noskip / fw3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for n in ${TEST_LIBS:-base fw3}; do
  lib=phase-vocoder_amd/build/libpv.so; [ $n != base ] && lib=phase-vocoder_amd/build/variants/libpv_$n.so
  PV_LIB_PATH=$PWD/$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ab/skip_tests_$n.log 2>&1
  rc=$?; echo "tests $n rc=$rc: $(tail -1 gpurun_out/ab/skip_tests_$n.log)"
  [ $rc -ne 0 ] && { grep -E "assert|Error|FAILED" gpurun_out/ab/skip_tests_$n.log | head -8; exit $rc; }
done
AB_ARGS="--workload c2" AB_STEPS=400 bash scripts/ab.sh ${AB_LIBS:-noskip fw3} || exit $?
