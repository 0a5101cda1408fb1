set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_fused_tests.log 2>&1 || { tail -30 gpurun_out/r05_fused_tests.log; exit 1; }
tail -2 gpurun_out/r05_fused_tests.log
for a in "" "--write-spec"; do
  timeout -k 10 200 python bench.py --workload c2 --no-cpu $a > gpurun_out/r05_c2$a.log 2>&1 || exit 1
  python3 -c "
import json,sys
d=json.loads([l for l in open('gpurun_out/r05_c2$a.log') if l.startswith('{')][-1])
print('$a', d['value'], d['kernels'], d['roofline']['frac'], d['roofline']['bound'], d['config']['spectrum'], d['rms_vs_oracle']['max'])"
done
PV_LIB_PATH=$PWD/phase-vocoder_amd/build/variants/libpv_stamps.so timeout -k 10 120 python scripts/fused_stamps.py > gpurun_out/r05_stamps_nospec.json || exit 1
STAMPS_WRITE_SPEC=1 PV_LIB_PATH=$PWD/phase-vocoder_amd/build/variants/libpv_stamps.so timeout -k 10 120 python scripts/fused_stamps.py > gpurun_out/r05_stamps_spec.json || exit 1
cut -c1-700 gpurun_out/r05_stamps_nospec.json gpurun_out/r05_stamps_spec.json
