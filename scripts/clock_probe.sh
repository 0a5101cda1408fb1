#!/bin/bash
# Sample the GPU's shader clock and power while bench.py runs a long timed loop:
# tells whether the kernels run power/clock limited.  Diagnostic only.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 python bench.py --no-cpu --steps ${STEPS:-400} --warmup 3 ${BENCH_ARGS:-} > gpurun_out/clock_bench.log 2>&1 &
pid=$!
sleep ${DELAY:-12}
for i in $(seq 1 ${SAMPLES:-10}); do
  rocm-smi --showclocks --showpower 2>/dev/null | grep -E "sclk|fclk|mclk|Power" | tr -s ' ' | head -8
  echo "--"
  sleep 0.5
done > gpurun_out/clock_samples.log
wait $pid
echo "bench rc=$?"
grep '^{' gpurun_out/clock_bench.log | cut -c1-200
head -40 gpurun_out/clock_samples.log
