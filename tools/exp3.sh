set -e
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -x -q -k gemm > gpurun_out/kern.log 2>&1 || { tail -20 gpurun_out/kern.log; exit 1; }
tail -1 gpurun_out/kern.log
timeout -k 10 200 python tools/gemm_tune.py --variants 8,13,14,21,22,23 2>/dev/null | grep -v amdgpu
run() { echo "== var=$1"; CLIPVIT_GEMM_VARIANTS=$1 timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --profile-iters 1 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['ms_per_step'], d['roofline']['family_ms_per_forward'])"; }
run 8,14,13,14,14; run 21,21,21,21,21; run 8,21,21,21,21; run 21,21,13,21,21; run 23,21,21,21,21
