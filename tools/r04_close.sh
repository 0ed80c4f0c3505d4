set -o pipefail
bash tools/gpu_tests.sh || exit 1
mkdir -p gpurun_out/c21
timeout -k 10 400 python -u bench.py > gpurun_out/c21/default.json 2> gpurun_out/c21/default.err || { echo "bench failed"; tail -20 gpurun_out/c21/default.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/c21/default.json'));print(d['value'], d['roofline']['frac'], d['parity']['max_rel_logit_err_vs_cpu_fp32_oracle'])"
