#!/usr/bin/env bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
bash tools/gpu_ab.sh "FSCNN_TMP_ORDER=0" "FSCNN_TMP_ORDER=1"
bash tools/gpu_ab.sh "FSCNN_TMP_ORDER=0" "FSCNN_TMP_ORDER=1"
