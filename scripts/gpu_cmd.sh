set -u
mkdir -p gpurun_out
STEPS="tests c3 c2 c4 compat rt prof prof_c4 prof_c2 prof_compat" bash scripts/round_evidence.sh || exit $?
echo all done
