# MX variant 4 (gemm_p32mx.h): kernel tests, kernel A/B against variant 3, config-5 in-model A/B
set -o pipefail
out=gpurun_out/r06_mx
mkdir -p $out
case "${1:-all}" in
  all)
    timeout -k 10 400 python -u -m pytest tests/test_gpu_mx8.py -x -v --timeout 200 --timeout-method thread -k "p32" > $out/tests.log 2>&1 || { echo "tests failed"; tail -40 $out/tests.log; exit 1; }
    grep -E "PASSED|FAILED|passed|failed" $out/tests.log | tail -12
    GEMM_AB_DTYPE=3 timeout -k 10 300 python -u tools/gemm_ab.py "12800,3072,768,1;12800,2304,768,0;25600,3072,768,1;25600,2304,768,0" "3,4,3403,3404" 5 20 > $out/gemm_ab.log 2>&1 || { echo "gemm_ab failed"; tail -10 $out/gemm_ab.log; exit 1; }
    cat $out/gemm_ab.log
    timeout -k 10 900 bash tools/ab_envs.sh "--dtype mxfp8 --batch 512 --steps 20 --warmup 5" 2 - "--tuning mx8_variants=4,5,4,3" "--tuning mx8_variants=4,5,3,3" > $out/ab.log 2>&1 || { echo "A/B failed"; tail -20 $out/ab.log; exit 1; }
    cat $out/ab.log ;;
  fc)
    timeout -k 10 1000 bash tools/ab_envs.sh "--dtype mxfp8 --batch 512 --steps 20 --warmup 5" 2 - "--tuning mx8_variants=3,5,4,3" "--tuning split_min=0" "--tuning mx8_variants=3,5,4,3;split_min=0" > $out/ab_fc.log 2>&1 || { echo "A/B failed"; tail -20 $out/ab_fc.log; exit 1; }
    cat $out/ab_fc.log ;;
esac
