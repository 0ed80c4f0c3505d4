set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mx8.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gemm" > gpurun_out/mx_t.log 2>&1 || { echo "mx tests failed"; tail -40 gpurun_out/mx_t.log; exit 1; }
tail -1 gpurun_out/mx_t.log
timeout -k 10 300 python -u tools/gemm_tune.py --batch 512 --dtype 3 --variants 2,202,3402,3,203,3403,4,204,3404 --iters 30 || exit 1
for v in "2,2,2,2" "3,3,3,3" "203,203,203,203"; do
  CLIPVIT_MX8_VARIANTS=$v timeout -k 10 300 python -u bench.py --dtype mxfp8 --batch 512 --no-cpu-baseline > gpurun_out/ab.json 2> gpurun_out/ab.err || { echo "bench failed $v"; tail -5 gpurun_out/ab.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/ab.json')); f=d['roofline']['family_ms_per_forward']
print('$v', round(d['value']), 'img/s', ' '.join(f'{k}={v:.3f}' for k,v in f.items()), 'parity', d['parity'], flush=True)"
done
