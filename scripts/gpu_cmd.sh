set -u
mkdir -p gpurun_out
STEPS="tests" bash scripts/round_evidence.sh || exit $?
echo all done
