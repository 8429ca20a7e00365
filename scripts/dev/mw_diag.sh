cd "$GRAFT_REPO_ROOT"; export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 200 python scripts/dev/mw_diag.py
