#!/usr/bin/env bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
bash tools/gpu_ab.sh "FSCNN_TMP_INK=15" "FSCNN_TMP_INK=14" "FSCNN_TMP_INK=13" "FSCNN_TMP_INK=11" "FSCNN_TMP_INK=7" "FSCNN_TMP_INK=0"
