mkdir -p gpurun_out/exp2
run() { echo "== split=$1 var=$2"; CLIPVIT_SPLIT_MIN=$1 CLIPVIT_GEMM_VARIANTS=$2 timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --profile-iters 1 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['ms_per_step'])"; }
run 0 8,14,13,14,14 && run 64 8,14,13,14,14 && run 0 15,14,15,14,14 && run 64 15,14,15,14,14 && run 64 13,13,13,13,13 && run 64 11,11,11,11,11 && run 0 13,13,13,13,13 && run 64 7,7,7,7,7
