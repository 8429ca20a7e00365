#!/bin/bash
# One entry point for the GPU-box work (run through gpurun). Every GPU step has its own time
# limit and the script stops at the first failure.
#   scripts/gpu.sh tests [pytest -k expr]        GPU test suite, then smoke()
#   scripts/gpu.sh files FILE...                  selected GPU test files
#   scripts/gpu.sh bench [N] [STEPS] [WARM] [REPS]  bench.py runs -> gpurun_out/bench.jsonl
#   scripts/gpu.sh rehearse [N] [STEPS] [WARM]   N ranks on the one GPU: SPMD self-launch (gloo
#                                                 bootstrap, xGMI gradients) + estimator topology
#   scripts/gpu.sh prof NAME CMD...              rocprofv3 kernel trace + stats -> gpurun_out/prof/NAME
#   scripts/gpu.sh pmc PASS bench|lin            one PMC counter pass (1..3) -> gpurun_out/pmc
#   scripts/gpu.sh dlrm [BATCH...]               DLRM train bench (graph + eager) -> gpurun_out/dlrm.jsonl
#   scripts/gpu.sh e2e                           DLRM end-to-end bench (1/2 workers) -> gpurun_out/dlrm_e2e.jsonl
#   scripts/gpu.sh trace [N]                     span timeline of the estimator topology, N workers on the
#                                                 one GPU (RAYDP_TRACE) -> gpurun_out/tr, *_timeline.txt
#   scripts/gpu.sh xgmi [WORLD...]               one-shot xGMI collective bench, ranks share the GPU
#   scripts/gpu.sh warm [WARM] [RUNS]            headline pipeline: per-run walls/phases after warm-up
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
T="python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider"
cmd=$1; shift
case $cmd in
  tests)
    K=${1:+-k "$1"}
    timeout -k 10 900 $T tests/ -m gpu $K > gpurun_out/gpu_tests.log 2>&1
    rc=$?; echo "gpu tests rc=$rc"; grep -E "passed|failed|^E  " gpurun_out/gpu_tests.log | tail -15
    [ $rc -ne 0 ] && exit $rc
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
    rc=$?; tail -1 gpurun_out/smoke.log; exit $rc;;
  files)
    # selected GPU test files (no smoke): scripts/gpu.sh files tests/test_gpu_xgmi.py ...
    timeout -k 10 1000 $T "$@" -m gpu > gpurun_out/gpu_files.log 2>&1
    rc=$?; echo "gpu files rc=$rc"; grep -E "passed|failed|^E  |PASSED|FAILED" gpurun_out/gpu_files.log | tail -40
    exit $rc;;
  bench)
    N=${1:-1}; S=${2:-20}; W=${3:-5}; REPS=${4:-3}
    for i in $(seq $REPS); do
      timeout -k 10 300 python bench.py --gpus $N --steps $S --warmup $W >> gpurun_out/bench.jsonl 2>> gpurun_out/bench.err || exit 9
    done
    tail -c 1500 gpurun_out/bench.jsonl;;
  rehearse)
    N=${1:-2}; S=${2:-20}; W=${3:-5}
    RAYDP_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus $N --steps $S --warmup $W \
      >> gpurun_out/rehearse_spmd.jsonl 2>> gpurun_out/rehearse.err || exit 12
    timeout -k 10 300 python bench.py --gpus $N --gpu-share $(python -c "print(1/$N)") --topology estimator \
      --steps $S --warmup $W >> gpurun_out/rehearse_estimator.jsonl 2>> gpurun_out/rehearse.err || exit 13
    tail -c 900 gpurun_out/rehearse_spmd.jsonl; tail -c 900 gpurun_out/rehearse_estimator.jsonl;;
  prof)
    NAME=$1; shift
    mkdir -p gpurun_out/prof
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof/$NAME -o run \
      -- "$@" > $R/gpurun_out/prof/$NAME.log 2>&1
    rc=$?; echo "prof rc=$rc"; exit $rc;;
  pmc)
    mkdir -p gpurun_out/pmc
    cd /tmp && export TMPDIR=/tmp
    case $1 in
      1) P="SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE";;
      2) P="FETCH_SIZE TCC_HIT_sum SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES";;
      3) P="WRITE_SIZE TCC_MISS_sum SQ_INSTS_VALU SQ_INSTS_SALU";;
      *) echo "pass 1..3"; exit 2;;
    esac
    REGEX="rx_jit_persist|rx_jit_step_mw|opt_tiled|mlp_persist|lin_gemm|arrow_ingest|xg_allreduce|mt_sgd"
    if [ "$2" = bench ]; then
      CMD="python3 $R/bench.py --steps 200 --warmup 5 --no-reference-config --extra-workloads none"
    elif [ "$2" = mw ]; then
      CMD="python3 $R/bench.py --rows 400000 --epochs 1 --batch 4096 --steps 20 --warmup 5 --extra-workloads none"
    else
      CMD="python3 $R/benchmarks/linear_gemm_bench.py --reps 3"
    fi
    timeout -s KILL 150 rocprofv3 --pmc $P --kernel-include-regex "$REGEX" --output-format csv \
      -d $R/gpurun_out/pmc -o $2_p$1 -- $CMD > $R/gpurun_out/pmc/$2_p$1.log 2>&1
    rc=$?; echo "pmc rc=$rc"; exit $rc;;
  dlrm)
    for B in ${@:-2048 128}; do
      timeout -k 10 200 python benchmarks/dlrm_bench.py --batch $B --steps 400 --warmup 40 --graph \
        >> gpurun_out/dlrm.jsonl 2>> gpurun_out/dlrm.err || exit 14
      timeout -k 10 200 python benchmarks/dlrm_bench.py --batch $B --steps 400 --warmup 40 \
        >> gpurun_out/dlrm.jsonl 2>> gpurun_out/dlrm.err || exit 15
    done
    cat gpurun_out/dlrm.jsonl;;
  e2e)
    # DLRM end to end (synthetic Criteo TSV -> preprocessing -> fit_on_spark): the notebook's
    # batch 128 with 1 and 2 workers, and batch 2048 with 1 worker
    for cfg in "128 50000 5000 2" "128 50000 5000 1" "2048 200000 20000 1"; do
      set -- $cfg
      timeout -k 10 400 python benchmarks/dlrm_e2e_bench.py --batch $1 --rows $2 --warmup-rows $3 --workers $4 \
        >> gpurun_out/dlrm_e2e.jsonl 2>> gpurun_out/dlrm_e2e.err || exit 16
    done
    cut -c1-400 gpurun_out/dlrm_e2e.jsonl;;
  trace)
    N=${1:-2}
    mkdir -p gpurun_out/tr; rm -f gpurun_out/tr/est.*
    RAYDP_TRACE=gpurun_out/tr/est timeout -k 10 300 python bench.py --gpus $N --gpu-share $(python -c "print(1/$N)") \
      --topology estimator --steps 20 --warmup 5 --no-reference-config > gpurun_out/trace_est.jsonl \
      2> gpurun_out/trace_est.err || exit 17
    python scripts/trace_summary.py gpurun_out/tr/est > gpurun_out/trace_est_timeline.txt 2>&1
    head -60 gpurun_out/trace_est_timeline.txt;;
  xgmi)
    for W in ${@:-4 8}; do
      timeout -k 10 300 python benchmarks/xgmi_bench.py --world $W >> gpurun_out/xgmi.jsonl \
        2>> gpurun_out/xgmi.err || exit 18
    done
    cat gpurun_out/xgmi.jsonl;;
  warm)
    timeout -k 10 300 python scripts/dev/warm_gap.py --warm ${1:-3,2} --runs ${2:-8} >> gpurun_out/warm_gap.jsonl \
      2>> gpurun_out/warm_gap.err || exit 19
    cut -c1-300 gpurun_out/warm_gap.jsonl;;
  *) echo "usage: scripts/gpu.sh tests|bench|rehearse|prof|pmc|dlrm|e2e|trace|xgmi|warm ..."; exit 2;;
esac
