#!/bin/bash
# Evidence run for the judged numbers: GPU tests, the bench lines (c3 headline with the CPU
# baseline, c2, c4, compat, rt), the rocprofv3 kernel-trace summaries of the bench commands
# and the FETCH/WRITE passes for profiles/traffic.json.  Stops at the first failing GPU step.
#   STEPS="tests c3 prof" bash scripts/round_evidence.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name seconds cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; grep '^{' gpurun_out/$name.log | tail -1 | cut -c1-600
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/$name.log; exit $rc; fi
}
prof() {  # name seconds bench-args...  (the program right after --)
  local name=$1 t=$2; shift 2
  rm -rf gpurun_out/$name
  run $name $t rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$name -o run -- python3 bench.py "$@"
}
STEPS="${STEPS:-tests c3 c2 c4 compat rt prof pmc}"
for s in $STEPS; do
  case $s in
    probe3) run valu_probe3 300 scripts/valu_probe3 ;;
    tests) run pytest_gpu 700 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread ${PYTEST_ARGS:-}; tail -3 gpurun_out/pytest_gpu.log ;;
    c3) run bench_c3 400 python bench.py ;;
    c3q) run bench_c3 300 python bench.py --no-cpu ;;
    c2) run bench_c2 300 python bench.py --workload c2 ;;
    c4) run bench_c4 300 python bench.py --workload c4 --no-cpu ;;
    compat) run bench_compat 300 python bench.py --workload compat ;;
    rt) run bench_rt 300 python bench.py --workload rt ;;
    prof) prof prof 400 --steps 40 --warmup 3 --no-cpu ;;
    prof_c4) prof prof_c4 400 --workload c4 --steps 40 --warmup 3 --no-cpu ;;
    prof_compat) prof prof_compat 400 --workload compat --steps 20 --warmup 3 --no-cpu ;;
    prof_c2) prof prof_c2 400 --workload c2 --no-cpu ;;
    traffic_c3|traffic_c4|traffic_c2)
      w=${s#traffic_}; rm -rf gpurun_out/pmc
      args="--calib"; [ $w = c4 ] && args="--calib --N 2048 --effect p --scale 1.5"
      [ $w = c2 ] && args="--calib --channels 1 --n 2646000 --effect p --scale 2.0 --reps 20"
      PV_TRAFFIC_WORKLOAD=$w PMC_SETS=scripts/pmc_sets_traffic.txt PROF_ARGS="$args" timeout -k 10 400 bash scripts/pmc_session.sh > gpurun_out/pmc_$w.log 2>&1
      rc=$?; tail -3 gpurun_out/pmc_$w.log; [ $rc -ne 0 ] && exit $rc
      rm -rf gpurun_out/pmc_$w && mv gpurun_out/pmc gpurun_out/pmc_$w ;;
    pmc)
      rm -rf gpurun_out/pmc
      PMC_SETS=scripts/pmc_sets_r1.txt PROF_ARGS="--calib" timeout -k 10 900 bash scripts/pmc_session.sh > gpurun_out/pmc_session.log 2>&1
      rc=$?; tail -8 gpurun_out/pmc_session.log; [ $rc -ne 0 ] && exit $rc
      python3 scripts/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc/summary.txt ;;
  esac
done
echo "evidence done"
