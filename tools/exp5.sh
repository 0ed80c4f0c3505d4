mkdir -p gpurun_out
( timeout -k 10 200 python bench.py --steps 12000 --warmup 5 --no-cpu-baseline --profile-iters 1 > gpurun_out/bench_long.log 2>&1 ) &
BP=$!
sleep 22
for i in 1 2 3; do amd-smi metric -g 0 --clock --power 2>&1 | head -40; echo ---; sleep 2; done > gpurun_out/smi.log 2>&1
wait $BP
tail -1 gpurun_out/bench_long.log | cut -c1-200
