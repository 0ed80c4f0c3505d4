set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py tests/test_gpu_mx8.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/lib_t.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/lib_t.log; exit 1; }
tail -1 gpurun_out/lib_t.log
NEW=$PWD/ai-interior-image-classifier_amd/libclipvit_hip.so; OLD=$PWD/ab/base.so
bash tools/ab_env.sh "" CLIPVIT_LIB "$OLD $NEW" 3 || exit 1
bash tools/ab_env.sh "--model ViT-B/16" CLIPVIT_LIB "$OLD $NEW" 2 || exit 1
bash tools/ab_env.sh "--model ViT-L/14@336px --batch 128 --lora-rank 16 --steps 5 --warmup 2" CLIPVIT_LIB "$OLD $NEW" 1
