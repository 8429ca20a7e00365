# DLRM persistent step: numerics tests, then the batch-128 bench at several grid sizes, the
# launch-per-op graph baseline on the same box, a rocprof kernel-stats pass; MW dump first.
cd "$GRAFT_REPO_ROOT"; export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 200 python scripts/dev/mw_dump.py > gpurun_out/mw_dump.txt 2>&1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_dlrm_step.py \
  > gpurun_out/dlrm_step_tests.txt 2>&1 && \
for G in 32 64 128; do
  RAYDP_DLRM_STEP_G=$G timeout -k 10 120 python benchmarks/dlrm_bench.py --persistent --batch 128 --steps 400 --warmup 16 \
    >> gpurun_out/dlrm_step_bench.jsonl 2>> gpurun_out/dlrm_step_bench.err || exit 1
done && \
timeout -k 10 180 python benchmarks/dlrm_bench.py --batch 128 --steps 400 --warmup 16 --graph \
  >> gpurun_out/dlrm_step_bench.jsonl 2>> gpurun_out/dlrm_step_bench.err && \
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
RAYDP_DLRM_STEP_G=64 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dlrm_step -o run -- \
  python benchmarks/dlrm_bench.py --persistent --batch 128 --steps 200 --warmup 16 > gpurun_out/dlrm_step_prof.log 2>&1
echo "exit $?"
