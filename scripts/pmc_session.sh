#!/bin/bash
# Counter passes (each its own rocprofv3 run; --pmc never combined with trace domains).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
i=0
while IFS= read -r set; do
  [ -z "$set" ] && continue
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-include-regex "pv::" --pmc $set --output-format csv -d gpurun_out/pmc/p$i -o run -- python3 scripts/prof_kernels.py ${PROF_ARGS:-} > gpurun_out/pmc/p$i.log 2>&1
  rc=$?; echo "pass $i ($set) rc=$rc"
  case $rc in 124|134|137|139) echo FATAL; exit $rc;; esac
done < "${PMC_SETS:-scripts/pmc_sets.txt}"
echo pmc done
