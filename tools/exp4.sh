set -e
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -x -q -k gemm > gpurun_out/kern.log 2>&1 || { tail -30 gpurun_out/kern.log; exit 1; }
tail -1 gpurun_out/kern.log
timeout -k 10 200 python tools/gemm_tune.py --variants 8,21,24,25,26,27 2>/dev/null | grep -v amdgpu
run() { echo "== var=$1"; CLIPVIT_GEMM_VARIANTS=$1 timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --profile-iters 1 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['ms_per_step'], d['roofline']['family_ms_per_forward'])"; }
run 8,21,21,21,21; run 24,24,24,24,24; run 25,24,25,24,24; run 8,24,26,24,24; run 27,24,27,24,24
