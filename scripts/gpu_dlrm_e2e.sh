# DLRM end to end through the Spark path (BASELINE config 5): plain and fused-SGD, plus one
# traced run (span timeline of the timed region).
set -o pipefail
mkdir -p gpurun_out/dtr
timeout -k 10 300 python benchmarks/dlrm_e2e_bench.py --rows 200000 --epochs 2 --batch 2048 > gpurun_out/dlrm_e2e.log 2>&1 || exit 1
timeout -k 10 300 python benchmarks/dlrm_e2e_bench.py --rows 200000 --epochs 2 --batch 2048 --fused-sgd > gpurun_out/dlrm_e2e_fused_sgd.log 2>&1 || exit 1
RAYDP_TRACE=gpurun_out/dtr/d timeout -k 10 300 python benchmarks/dlrm_e2e_bench.py --rows 200000 --epochs 2 --batch 2048 > gpurun_out/dlrm_e2e_traced.log 2>&1 || exit 1
python scripts/trace_summary.py gpurun_out/dtr/d | grep -v "chain input" > gpurun_out/dlrm_timeline.txt
