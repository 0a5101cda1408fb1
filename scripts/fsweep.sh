cd $GRAFT_REPO_ROOT
for rep in 1 2; do for f in 32 48 64 96; do
  PV_RUN_FRAMES=$f timeout -k 10 200 python bench.py --no-cpu > gpurun_out/f$f.log 2>&1 || exit 1
  python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/f$f.log') if l.startswith('{')][0]
print('F=$f', '%.4g' % d['value'], ' '.join('%s=%.3f' % (k, v['avg_ms']) for k, v in d['kernels'].items()))"
done; done
