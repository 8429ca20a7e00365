# DLRM phase profile, then headline cProfile + timeline, then the multi-workgroup NYC suite/bench
cd "$GRAFT_REPO_ROOT"; export HSA_ENABLE_IPC_MODE_LEGACY=0; mkdir -p gpurun_out
bash scripts/dev/r4_dlrm_phase.sh || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --extra-workloads none --profile-timed gpurun_out/headline_cprof.txt \
  > gpurun_out/headline.jsonl 2> gpurun_out/headline.err || exit 2
RAYDP_TRACE=gpurun_out/tr/h timeout -k 10 300 python bench.py --steps 20 --warmup 5 --extra-workloads none \
  >> gpurun_out/headline.jsonl 2>> gpurun_out/headline.err || exit 3
python scripts/trace_summary.py gpurun_out/tr/h > gpurun_out/headline_timeline.txt 2>&1
bash scripts/dev/r4_gpu_mw.sh
