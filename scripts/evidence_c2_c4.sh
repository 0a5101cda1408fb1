set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c2 -o run -- python3 bench.py --workload c2 --no-cpu > gpurun_out/prof_c2.log 2>&1 || exit $?
echo c2 prof done
PMC_SETS=scripts/pmc_sets_r1.txt PROF_ARGS="--N 2048 --effect p --scale 1.5" timeout -k 10 600 bash scripts/pmc_session.sh > gpurun_out/pmc_session.log 2>&1 || exit $?
tail -3 gpurun_out/pmc_session.log
python3 scripts/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc/summary_c4.txt
echo done
