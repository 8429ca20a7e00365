#!/bin/bash
# Full GPU check: kernel/engine tests -> smoke -> bench -> 2-rank rehearsal -> rocprof kernel stats.
# Every GPU step has its own time limit; the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out/prof
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; grep -E "passed|failed|^E  |Error" gpurun_out/gpu_tests.log | tail -15
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/smoke.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
RAYDP_BENCH_BACKEND=gloo RAYDP_BENCH_CPUS=2 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 1000 --warmup 100 > gpurun_out/bench2_gloo.log 2>&1
rc=$?; echo "bench2 rc=$rc"; grep metric gpurun_out/bench2_gloo.log | tail -1
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o bench -- python3 $R/bench.py --steps 1000 --warmup 100 > $R/gpurun_out/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -1 $R/gpurun_out/prof.log
find $R/gpurun_out/prof -name "*stats*"
exit $rc
