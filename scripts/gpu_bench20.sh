# 20-step driver-config bench, three back-to-back runs, then one traced run (span timeline
# of the timed region: scripts/trace_summary.py) and the no-flag default bench.
set -o pipefail
mkdir -p gpurun_out/tr
timeout -k 10 300 python -u -m pytest tests/test_gpu_xgmi.py -x -q --timeout 120 --timeout-method thread > gpurun_out/xgmi_tests.log 2>&1 || exit 1
for k in 1 2 3; do timeout -k 10 180 python bench.py --gpus 1 --steps 20 --warmup 5 --no-reference-config > gpurun_out/b20_fused_$k.log 2>&1 || exit 1; done
RAYDP_TRACE=gpurun_out/tr/nyc timeout -k 10 180 python bench.py --gpus 1 --steps 20 --warmup 5 --no-reference-config > gpurun_out/b20_traced.log 2>&1 || exit 1
python scripts/trace_summary.py gpurun_out/tr/nyc > gpurun_out/b20_timeline.txt || exit 1
timeout -k 10 240 python bench.py > gpurun_out/bench_default.log 2>&1
