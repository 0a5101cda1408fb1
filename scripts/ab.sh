#!/bin/bash
# A/B of libpv variants on one GPU box: bench.py (no CPU leg, no check) per variant, kernel
# times, two repetitions interleaved.
# usage: bash scripts/ab.sh [variant ...]
#   variant = <lib>[:VAR=value[,VAR=value...]]   lib: "base" (build/libpv.so) or the name of
#   build/variants/libpv_<name>.so; the optional environment is set for that run only
#   (e.g. base:PV_RUN_FRAMES=64).  Default: every build/variants/libpv_*.so.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
names=("$@")
if [ ${#names[@]} -eq 0 ]; then
  for f in phase-vocoder_amd/build/variants/libpv_*.so; do n=$(basename "$f" .so); names+=("${n#libpv_}"); done
fi
for rep in 1 2; do
  for v in base "${names[@]}"; do
    n=${v%%:*}; envs=""; [ "$v" != "$n" ] && envs=${v#*:}
    if [ "$n" = base ]; then lib=phase-vocoder_amd/build/libpv.so; else lib=phase-vocoder_amd/build/variants/libpv_$n.so; fi
    tag=$(echo "$v" | tr ':,=/' '____')
    env PV_LIB_PATH=$PWD/$lib ${envs//,/ } timeout -k 10 240 python bench.py --no-cpu --no-check --steps ${AB_STEPS:-10} ${AB_ARGS:-} > gpurun_out/ab/$tag.$rep.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "$v rc=$rc"; tail -3 gpurun_out/ab/$tag.$rep.log; exit $rc; fi
    python3 -c "
import json
l=[x for x in open('gpurun_out/ab/$tag.$rep.log') if x.startswith('{')][0]; d=json.loads(l)
print('%-28s rep$rep value=%.4g ' % ('$v', d['value']) + ' '.join('%s=%.4f' % (k, v['avg_ms']) for k, v in d['kernels'].items()))"
  done
done
