#!/bin/bash
# A/B of libpv variants on one GPU box: bench.py (no CPU leg) per variant, kernel times.
# usage: bash scripts/ab.sh [variant names...]   (default: every build/variants/libpv_*.so)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
names=("$@")
if [ ${#names[@]} -eq 0 ]; then
  for f in phase-vocoder_amd/build/variants/libpv_*.so; do n=$(basename "$f" .so); names+=("${n#libpv_}"); done
fi
for rep in 1 2; do
  for n in base "${names[@]}"; do
    if [ "$n" = base ]; then lib=phase-vocoder_amd/build/libpv.so; else lib=phase-vocoder_amd/build/variants/libpv_$n.so; fi
    PV_LIB_PATH=$PWD/$lib timeout -k 10 240 python bench.py --no-cpu --no-check --steps ${AB_STEPS:-10} ${AB_ARGS:-} > gpurun_out/ab/$n.$rep.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "$n rc=$rc"; tail -3 gpurun_out/ab/$n.$rep.log; exit $rc; fi
    python3 -c "
import json,sys
l=[x for x in open('gpurun_out/ab/$n.$rep.log') if x.startswith('{')][0]; d=json.loads(l)
print('%-14s rep$rep value=%.4g ' % ('$n', d['value']) + ' '.join('%s=%.4f' % (k, v['avg_ms']) for k, v in d['kernels'].items()))"
  done
done
