#!/bin/bash
# Round 5: config 4 with the spectrum not handed back (bins 684..1024 of pitch 1.5 not
# analysed) vs --write-spec (every bin): parity tests, then bench c4 A/B, 2 repetitions.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ab/c4skip_tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/ab/c4skip_tests.log)"
[ $rc -ne 0 ] && { grep -E "assert|Error|FAILED" gpurun_out/ab/c4skip_tests.log | head -12; exit $rc; }
for rep in 1 2; do
  for a in "" "--write-spec"; do
    tag=c4${a:+_ws}.$rep
    timeout -k 10 240 python bench.py --workload c4 --no-cpu --no-check $a > gpurun_out/ab/$tag.log 2>&1 || { tail -5 gpurun_out/ab/$tag.log; exit 1; }
    python3 -c "
import json
l=[x for x in open('gpurun_out/ab/$tag.log') if x.startswith('{')][0]; d=json.loads(l)
print('%-12s value=%.4g ' % ('$tag', d['value']) + ' '.join('%s=%.4f' % (k, v['avg_ms']) for k, v in d['kernels'].items()))"
  done
done
