#!/bin/bash
# Round 5: raw per-wave stamps of the config-2 single launch (placement: hw id per wave),
# twice per mode, to see whether the wave -> SIMD placement is deterministic.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/place
for rep in 1 2; do for b in 1 0; do
  PV_FUSED_BALANCE=$b PV_LIB_PATH=$PWD/phase-vocoder_amd/build/variants/libpv_stamps.so timeout -k 10 120 python scripts/fused_stamps.py 2646000 gpurun_out/place/st_bal${b}_rep$rep.npy > gpurun_out/place/bal${b}_rep$rep.json || exit 1
done; done
echo done
