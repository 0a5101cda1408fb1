#!/bin/bash
# Evidence run for the judged numbers: GPU tests, the bench lines (c3 headline with the CPU
# baseline, c2, c4, rt), the rocprofv3 kernel-trace summary of the headline bench and the
# FETCH/WRITE passes for profiles/traffic.json.  Stops at the first failing GPU step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name seconds cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; grep '^{' gpurun_out/$name.log | tail -1 | cut -c1-400
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/$name.log; exit $rc; fi
}
STEPS="${STEPS:-tests c3 c2 c4 compat rt prof pmc}"
for s in $STEPS; do
  case $s in
    tests) run pytest_gpu 700 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread; tail -3 gpurun_out/pytest_gpu.log ;;
    c3) run bench_c3 400 python bench.py ;;
    c2) run bench_c2 300 python bench.py --workload c2 ;;
    c4) run bench_c4 300 python bench.py --workload c4 --no-cpu ;;
    compat) run bench_compat 300 python bench.py --workload compat ;;
    rt) run bench_rt 300 python bench.py --workload rt ;;
    prof)
      rm -rf gpurun_out/prof
      run prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 40 --warmup 3 --no-cpu ;;
    pmc)
      rm -rf gpurun_out/pmc
      PMC_SETS=scripts/pmc_sets_r1.txt PROF_ARGS="--calib" timeout -k 10 900 bash scripts/pmc_session.sh > gpurun_out/pmc_session.log 2>&1
      rc=$?; tail -8 gpurun_out/pmc_session.log; [ $rc -ne 0 ] && exit $rc
      python3 scripts/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc/summary.txt ;;
  esac
done
echo "evidence done"
