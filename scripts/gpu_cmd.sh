set -u
mkdir -p gpurun_out
echo "# c3" && AB_STEPS=20 bash scripts/ab.sh notoff || exit $?
echo "# c4" && AB_STEPS=20 AB_ARGS="--workload c4" bash scripts/ab.sh notoff || exit $?
echo all done
