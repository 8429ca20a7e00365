set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_resume.py tests/test_gpu_front.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_k.log 2>&1 || exit 1
bash scripts/gpu_bench20.sh
