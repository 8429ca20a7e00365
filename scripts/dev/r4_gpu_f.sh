# Collective thresholds and DDP bucket sizing, ranks sharing the one GPU:
#  1. one-shot vs two-shot xGMI all-reduce at 256 KiB / 1 / 4 / 16 MiB, world 2 and 4
#  2. the DDP bucket-size x comm-stream sweep on DLRM (scripts/dev/ddp_sweep.sh) + overlap trace
cd "$GRAFT_REPO_ROOT"; export HSA_ENABLE_IPC_MODE_LEGACY=0; mkdir -p gpurun_out
S=262144,1048576,4194304,16777216
for W in 2 4; do
  timeout -k 10 240 python benchmarks/xgmi_bench.py --world $W --sizes $S --reps 100 --kernel oneshot \
    >> gpurun_out/xgmi_ab.jsonl 2>> gpurun_out/xgmi_ab.err || exit 1
  timeout -k 10 240 python benchmarks/xgmi_bench.py --world $W --sizes $S --reps 100 --kernel twoshot \
    >> gpurun_out/xgmi_ab.jsonl 2>> gpurun_out/xgmi_ab.err || exit 2
done
cut -c1-600 gpurun_out/xgmi_ab.jsonl
bash scripts/dev/ddp_sweep.sh || exit 3
python scripts/trace_overlap.py gpurun_out/prof/ddp_overlap/run --kernel lin_ --with xg_allreduce > gpurun_out/ddp_overlap.txt 2>&1
cat gpurun_out/ddp_overlap.txt | head -30
