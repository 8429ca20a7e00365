cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/b1.jsonl 2> gpurun_out/b1.err || { echo b1 failed; tail -30 gpurun_out/b1.err; exit 1; }
cut -c1-3000 gpurun_out/b1.jsonl
timeout -k 10 400 python bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/b2.jsonl 2> gpurun_out/b2.err || { echo b2 failed; tail -30 gpurun_out/b2.err; exit 1; }
cut -c1-3000 gpurun_out/b2.jsonl
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --extra-workloads none > gpurun_out/b2t.jsonl 2> gpurun_out/b2t.err || { echo b2t failed; tail -30 gpurun_out/b2t.err; exit 1; }
cut -c1-1500 gpurun_out/b2t.jsonl
