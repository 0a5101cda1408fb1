#!/bin/bash
# Round 5: correctness + A/B of the analysis input-ring variants (built beforehand with
# `make variant`): bit-exact analysis and process parity per variant, then bench A/B.
# usage: bash scripts/r05_ring_ab.sh variant...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for v in "$@"; do
  lib=$PWD/phase-vocoder_amd/build/variants/libpv_$v.so
  PV_LIB_PATH=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 \
      --timeout-method thread -k "bit_exact or std_process_parity or multichannel" > gpurun_out/ab/test_$v.log 2>&1
  rc=$?
  tail -2 gpurun_out/ab/test_$v.log
  if [ $rc -ne 0 ]; then echo "variant $v tests rc=$rc"; exit $rc; fi
done
bash scripts/ab.sh "$@"
