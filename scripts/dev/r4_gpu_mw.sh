# Multi-workgroup fused MLP: numerics, then the single-workgroup regression suite, then bench
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 500 $T tests/test_gpu_mw.py -m gpu > gpurun_out/mw_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed|Error|assert" gpurun_out/mw_tests.log | tail -30; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 $T tests/test_gpu_kernels.py -m gpu > gpurun_out/kern_tests.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/kern_tests.log | tail -3; [ $rc -ne 0 ] && { grep -E "^E " gpurun_out/kern_tests.log | head; exit $rc; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --extra-workloads none > gpurun_out/mw_b1.jsonl 2> gpurun_out/mw_b1.err || exit 7
timeout -k 10 400 python bench.py --rows 2000000 --epochs 1 --batch 4096 --steps 20 --warmup 5 >> gpurun_out/mw_b1.jsonl 2>> gpurun_out/mw_b1.err || exit 8
timeout -k 10 400 python bench.py --rows 2000000 --epochs 1 --batch 1000 --steps 20 --warmup 5 >> gpurun_out/mw_b1.jsonl 2>> gpurun_out/mw_b1.err || exit 9
cut -c1-400 gpurun_out/mw_b1.jsonl; grep -o '"step_time_us[^}]*}\|"engine[^,]*\|"rank0_breakdown_s[^}]*}' gpurun_out/mw_b1.jsonl
