cd "${GRAFT_REPO_ROOT}"; export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_fused_optim.py tests/test_gpu_hvd.py > gpurun_out/r5_optim_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r5_optim_tests.log; [ $rc -ne 0 ] && { grep -E "^E  " gpurun_out/r5_optim_tests.log | head; exit $rc; }
RAYTRAIN_DEVICE=cuda timeout -k 10 300 python benchmarks/raytrain_bench.py > gpurun_out/r5_b4_gpu.jsonl 2> gpurun_out/r5_b4_gpu.err || { echo "b4 gpu rc=$?"; tail -5 gpurun_out/r5_b4_gpu.err; exit 2; }
tail -1 gpurun_out/r5_b4_gpu.jsonl | cut -c1-300
rm -f gpurun_out/r5_persist.jsonl
timeout -k 10 150 python -u scripts/dev/persist_ab.py . >> gpurun_out/r5_persist.jsonl 2>> gpurun_out/r5_persist.err || exit 3
tail -1 gpurun_out/r5_persist.jsonl | cut -c1-300
