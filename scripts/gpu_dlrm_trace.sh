set -o pipefail
mkdir -p gpurun_out/dtr
RAYDP_TRACE=gpurun_out/dtr/d timeout -k 10 300 python benchmarks/dlrm_e2e_bench.py --rows 200000 --epochs 2 --batch 2048 > gpurun_out/dlrm_e2e_traced.log 2>&1 || exit 1
python scripts/trace_summary.py gpurun_out/dtr/d > gpurun_out/dlrm_timeline.txt
