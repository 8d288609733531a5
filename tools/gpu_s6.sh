#!/usr/bin/env bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/diag_predict.py low > gpurun_out/diag_low.txt 2>&1; grep -v amdgpu.ids gpurun_out/diag_low.txt
