#!/bin/bash
# timing experiments of the persistent kernel (RAYDP_MLP_EXPERIMENT variants; numerics invalid)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for e in "" $@; do
  echo "== experiment '$e'"
  RAYDP_MLP_EXPERIMENT="$e" timeout -k 10 200 python -u scripts/dev/persist_time.py 1 2>&1 | grep -v amdgpu.ids || exit $?
done
