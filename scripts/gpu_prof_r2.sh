# rocprofv3 kernel statistics (CSV) of the headline bench at the driver config and the default.
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/prof20 $R/gpurun_out/prof3000
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof20 -o run -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-reference-config > $R/gpurun_out/prof20.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof3000 -o run -- python3 $R/bench.py --no-reference-config > $R/gpurun_out/prof3000.log 2>&1
