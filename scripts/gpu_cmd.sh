set -u
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
STEPS="tests c3 c2 c4 compat rt prof prof_c4 prof_c2 prof_compat" bash scripts/round_evidence.sh || exit $?
echo all done
