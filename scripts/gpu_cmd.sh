set -u
mkdir -p gpurun_out
STEPS="tests c3 c2 c4 compat rt prof prof_c4 prof_c2 prof_compat traffic_c3" bash scripts/round_evidence.sh || exit $?
timeout -k 10 120 phase-vocoder_amd/build/fft_bench bench > gpurun_out/fft_bench.log 2>&1 || exit $?
echo all done
