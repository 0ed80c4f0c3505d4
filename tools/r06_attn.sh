# persistent one-key-block attention (attn_persist): kernel + engine bit identity, then the B/32 A/B
set -o pipefail
out=gpurun_out/r06_attn
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -k "persistent" > $out/tests.log 2>&1 || { echo "tests failed"; tail -40 $out/tests.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $out/tests.log | tail -30
timeout -k 10 1000 bash tools/ab_envs.sh "--steps 20 --warmup 5" 2 - "--tuning attn_persist=1" "--tuning attn_persist=2" "--tuning attn_persist=3" > $out/ab.log 2>&1 || { echo "A/B failed"; tail -20 $out/ab.log; exit 1; }
cat $out/ab.log
