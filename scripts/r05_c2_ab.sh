#!/bin/bash
# Round 5: config-2 single launch A/B (bench c2 kernel time) + per-phase stamps of both
# builds.  usage: bash scripts/r05_c2_ab.sh variant... (stamps variants: stamps_<name>)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
AB_ARGS="--workload c2" AB_STEPS=${AB_STEPS:-200} bash scripts/ab.sh "$@" || exit $?
for s in ${STAMPS:-}; do
  PV_LIB_PATH=$PWD/phase-vocoder_amd/build/variants/libpv_$s.so timeout -k 10 120 python scripts/fused_stamps.py \
    > gpurun_out/ab/stamps_$s.json 2> gpurun_out/ab/stamps_$s.err || { echo "stamps $s failed"; tail -5 gpurun_out/ab/stamps_$s.err; exit 1; }
  echo "stamps $s: $(cut -c1-900 gpurun_out/ab/stamps_$s.json)"
done
