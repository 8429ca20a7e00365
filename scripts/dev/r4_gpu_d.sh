# Multi-workgroup fused MLP: numerics + kernel suite + batch 64/1000/4096 benches + rocprof at 4096
cd "$GRAFT_REPO_ROOT"; export HSA_ENABLE_IPC_MODE_LEGACY=0; mkdir -p gpurun_out/prof
R=$(pwd)
bash scripts/dev/r4_gpu_mw.sh || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof/mw4096 -o run -- \
  python3 $R/bench.py --rows 2000000 --epochs 1 --batch 4096 --steps 20 --warmup 5 --extra-workloads none \
  > $R/gpurun_out/prof/mw4096.log 2>&1 || { echo prof failed; tail -5 $R/gpurun_out/prof/mw4096.log; exit 1; }
head -6 $R/gpurun_out/prof/mw4096/run_kernel_stats.csv | cut -c1-250
