set -u
mkdir -p gpurun_out
STEPS="tests c3 c4 c2 compat prof prof_c4" bash scripts/round_evidence.sh || exit $?
AB_STEPS=20 AB_ARGS="--workload c4" bash scripts/ab.sh synfull || exit $?
PV_LIB_PATH=$PWD/phase-vocoder_amd/build/variants/libpv_stamps.so timeout -k 10 120 python scripts/fused_stamps.py > gpurun_out/r06_c2_stamps.json || exit $?
echo all done
