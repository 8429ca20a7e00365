# Data scale re-check after the executor inline-run / transport / CSV changes: 10 M rows at batch
# 64 and 4096 (8 executors), then DLRM end to end (batch 128 x 2 / x 1 workers, batch 2048)
cd "$GRAFT_REPO_ROOT"; export HSA_ENABLE_IPC_MODE_LEGACY=0; mkdir -p gpurun_out
rm -f gpurun_out/t_ds.jsonl gpurun_out/dlrm_e2e.jsonl
timeout -k 10 500 python bench.py --rows 10000000 --epochs 1 --batch 64 --steps 20 --warmup 5 >> gpurun_out/t_ds.jsonl 2> gpurun_out/t_ds.err || exit 1
timeout -k 10 400 python bench.py --rows 10000000 --epochs 1 --batch 4096 --steps 20 --warmup 5 >> gpurun_out/t_ds.jsonl 2>> gpurun_out/t_ds.err || exit 2
cut -c1-300 gpurun_out/t_ds.jsonl
bash scripts/gpu.sh e2e || exit 3
