#!/bin/bash
# Copy the judged results of a scripts/round_evidence.sh run (merged into gpurun_out/) into
# profiles/ under a round prefix: bench lines, rocprofv3 kernel stats, counter summary,
# GPU test log, and profiles/traffic.json from the FETCH/WRITE passes.
# usage: bash scripts/collect_evidence.sh r03
set -eu
cd "$(dirname "$0")/.."
r=${1:?round prefix, e.g. r03}
for w in c3 c2 c4 compat rt; do
  grep '^{' gpurun_out/bench_$w.log | tail -1 > profiles/${r}_bench_$w.json
done
grep '^{' gpurun_out/prof.log | tail -1 > profiles/${r}_bench_c3_under_rocprof.json
cp gpurun_out/prof/run_kernel_stats.csv profiles/${r}_kernel_stats.csv
cp gpurun_out/pmc/summary.txt profiles/${r}_pmc.txt
cp gpurun_out/pytest_gpu.log profiles/${r}_pytest_gpu.txt
python3 scripts/traffic_from_pmc.py gpurun_out/pmc profiles/traffic.json
echo "collected into profiles/${r}_*"
