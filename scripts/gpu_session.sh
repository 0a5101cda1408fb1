#!/bin/bash
# One GPU-box session: parity tests, bench, rocprof kernel trace.  Every GPU step has its
# own time limit; a fault / abort / timeout ends the session (no retries).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }

STEPS="${STEPS:-tests bench prof}"
for step in $STEPS; do
  case "$step" in
    tests)
      timeout -k 10 "${T_TESTS:-600}" python -m pytest tests -m gpu -q -rf ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
      rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_gpu.log
      if fatal $rc || [ $rc -gt 1 ]; then echo "FATAL in tests"; exit $rc; fi ;;
    rt)
      timeout -k 10 "${T_BENCH:-300}" python bench.py --workload rt > gpurun_out/bench_rt.log 2>&1
      rc=$?; echo "bench rt rc=$rc"; tail -3 gpurun_out/bench_rt.log
      if [ $rc -ne 0 ]; then echo "bench rt failed"; exit $rc; fi ;;
    fft)
      timeout -k 10 120 phase-vocoder_amd/build/fft_bench bench > gpurun_out/fft_bench.log 2>&1
      rc=$?; echo "fft bench rc=$rc"; cat gpurun_out/fft_bench.log
      if [ $rc -ne 0 ]; then exit $rc; fi ;;
    bench)
      timeout -k 10 "${T_BENCH:-600}" python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
      rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench.log
      if [ $rc -ne 0 ]; then echo "bench failed"; exit $rc; fi ;;
    prof)
      rm -rf gpurun_out/prof
      timeout -k 10 "${T_PROF:-600}" rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/prof.log 2>&1
      rc=$?; echo "prof rc=$rc"; tail -3 gpurun_out/prof.log
      find gpurun_out/prof -name "*stats*" | head
      if [ $rc -ne 0 ]; then exit $rc; fi ;;
    pmc)
      rm -rf gpurun_out/pmc_fetch gpurun_out/pmc_write
      timeout -k 10 "${T_PROF:-600}" rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/pmc_fetch.log 2>&1
      rc=$?; echo "pmc fetch rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc_fetch.log; exit $rc; fi
      timeout -k 10 "${T_PROF:-600}" rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/pmc_write.log 2>&1
      rc=$?; echo "pmc write rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc_write.log; exit $rc; fi ;;
  esac
done
echo "session done"
