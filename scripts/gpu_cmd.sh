set -u
mkdir -p gpurun_out
AB_STEPS=20 bash scripts/ab.sh saddr sawreg || exit $?
echo all done
