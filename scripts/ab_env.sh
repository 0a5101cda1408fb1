#!/bin/bash
# A/B of one environment switch on one GPU box: bench.py (no CPU leg), kernel times.
# usage: AB_VAR=PV_X AB_VALS="0 1" AB_WL="c3 c4" bash scripts/ab_env.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for wl in ${AB_WL:-c3}; do
    for v in ${AB_VALS:-0 1}; do
      log=gpurun_out/ab/$wl.$AB_VAR=$v.$rep.log
      env "$AB_VAR=$v" timeout -k 10 240 python bench.py --no-cpu --no-check --workload $wl ${AB_ARGS:-} > $log 2>&1
      rc=$?
      if [ $rc -ne 0 ]; then echo "$wl $v rc=$rc"; tail -3 $log; exit $rc; fi
      python3 -c "
import json
l=[x for x in open('$log') if x.startswith('{')][0]; d=json.loads(l)
print('%-4s %s=%s rep$rep value=%.4g ' % ('$wl', '$AB_VAR', '$v', d['value']) + ' '.join('%s=%.4f' % (k, v['avg_ms']) for k, v in d['kernels'].items()))"
    done
  done
done
