# MW reductions reworked: MW + kernel suites, rocprof at batch 4096, then data scale (8 executors)
cd "$GRAFT_REPO_ROOT"; export HSA_ENABLE_IPC_MODE_LEGACY=0; mkdir -p gpurun_out/prof
R=$(pwd)
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 500 $T tests/test_gpu_mw.py tests/test_gpu_kernels.py -m gpu > gpurun_out/mw_tests.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/mw_tests.log | tail -3; [ $rc -ne 0 ] && { grep -E "^E " gpurun_out/mw_tests.log | head; exit $rc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof/mw4096b -o run -- \
  python3 $R/bench.py --rows 2000000 --epochs 1 --batch 4096 --steps 20 --warmup 5 --extra-workloads none \
  > $R/gpurun_out/prof/mw4096b.log 2>&1 || { echo prof failed; tail -5 $R/gpurun_out/prof/mw4096b.log; exit 4; }
head -4 $R/gpurun_out/prof/mw4096b/run_kernel_stats.csv | cut -c1-160
cd $R && bash scripts/dev/r4_gpu_k.sh
