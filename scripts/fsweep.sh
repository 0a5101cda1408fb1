#!/bin/bash
# Frames-per-run sweep (PV_RUN_FRAMES) of one bench workload: FS="32 48 64" WL=c3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do for f in ${FS:-32 48 64 96}; do
  PV_RUN_FRAMES=$f timeout -k 10 200 python bench.py --no-cpu --workload ${WL:-c3} > gpurun_out/f$f.log 2>&1 || exit 1
  python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/f$f.log') if l.startswith('{')][0]
print('F=$f', '%.4g' % d['value'], ' '.join('%s=%.4f' % (k, v['avg_ms']) for k, v in d['kernels'].items()))"
done; done
