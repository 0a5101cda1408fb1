#!/bin/bash
# GPU parity tests against each variant library (PV_LIB_PATH), then scripts/ab.sh timing.
# Stops at the first failing variant.  usage: bash scripts/ab_tests.sh name...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for n in "$@"; do
  PV_LIB_PATH=$PWD/phase-vocoder_amd/build/variants/libpv_$n.so timeout -k 10 300 \
    python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/ab/tests_$n.log 2>&1
  rc=$?; echo "tests $n rc=$rc: $(tail -1 gpurun_out/ab/tests_$n.log)"
  if [ $rc -ne 0 ]; then grep -E "assert|Error|FAILED" gpurun_out/ab/tests_$n.log | head -8; exit $rc; fi
done
bash scripts/ab.sh "$@"
