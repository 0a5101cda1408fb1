#!/bin/bash
# A/B of the handle's own row layout (PV_ROW_LAYOUT=run vs natural) for c3 / c4, after the
# GPU suite with the run-major layout.  Stops at the first failing step.
# Needs scripts/r05_row_layout.patch applied (git apply) and the library rebuilt: PV_ROW_LAYOUT is not in the product.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != 1 ]; then
PV_ROW_LAYOUT=run timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/pytest_run.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_run.log; [ $rc -ne 0 ] && exit $rc
fi
for rep in 1 2; do
  for lay in natural run; do
    for w in c3 c4; do
      PV_ROW_LAYOUT=$lay timeout -k 10 200 python bench.py --workload $w --no-cpu --steps 30 --warmup 5 > gpurun_out/ab_${w}_${lay}_$rep.log 2>&1
      rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/ab_${w}_${lay}_$rep.log; exit $rc; }
      python3 - "$w" "$lay" "$rep" <<'PY'
import json,sys
d=[json.loads(l) for l in open(f"gpurun_out/ab_{sys.argv[1]}_{sys.argv[2]}_{sys.argv[3]}.log") if l.startswith('{')][-1]
kt=d.get('kernels')
print(sys.argv[1:], f"{d['value']:.4g}", f"{d['ms_per_step']:.4f}", d['roofline']['avg_launch_ms'], d['rms_vs_oracle']['max'], kt)
PY
    done
  done
done
