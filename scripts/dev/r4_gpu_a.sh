# xGMI collective tests (two-shot, comm stream, error word) + data-scale batch-4096 baseline
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_xgmi.py -m gpu > gpurun_out/xgmi_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/xgmi_tests.log | tail -30; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --rows 10000000 --epochs 1 --batch 64 --steps 20 --warmup 5 >> gpurun_out/ds2.jsonl 2> gpurun_out/ds2.err || { echo ds b64 failed; tail -20 gpurun_out/ds2.err; exit 1; }
timeout -k 10 400 python bench.py --rows 2000000 --epochs 1 --batch 4096 --steps 20 --warmup 5 >> gpurun_out/ds2.jsonl 2>> gpurun_out/ds2.err || { echo ds b4096 failed; tail -20 gpurun_out/ds2.err; exit 1; }
cut -c1-600 gpurun_out/ds2.jsonl; grep -o '"rank0_breakdown_s[^}]*}' gpurun_out/ds2.jsonl
