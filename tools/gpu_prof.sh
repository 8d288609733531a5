#!/usr/bin/env bash
# Round-3 profile set: rocprofv3 kernel stats + one-step trace of the bench train step, the
# per-layer HIP-event table, and the PMC HBM traffic of the dominant family.
#   tools/gpu_prof.sh <tag> [pmc]
set -uo pipefail
TAG=${1:-r03}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
bash tools/profile_step.sh ${TAG} --no-forward > gpurun_out/prof_${TAG}.txt 2>&1 || { tail -20 gpurun_out/prof_${TAG}.txt; exit 1; }
head -45 gpurun_out/prof_${TAG}.txt
TR=$(find gpurun_out/prof_${TAG} -name '*kernel_trace.csv' | head -1)
python3 tools/trace_step.py "$TR" --step 4 > gpurun_out/${TAG}_train_step_trace.txt || exit 1
tail -3 gpurun_out/${TAG}_train_step_trace.txt
FSCNN_SIDE_STREAM=0 timeout -k 10 300 python -u tools/layer_report.py gpurun_out/${TAG}_layers.md > gpurun_out/layers_${TAG}.log 2>&1 || { tail -20 gpurun_out/layers_${TAG}.log; exit 1; }
grep -A20 "kernel family" gpurun_out/${TAG}_layers.md | head -50
if [[ "${2:-}" == pmc ]]; then
  FSCNN_SIDE_STREAM=0 bash tools/pmc_step.sh ${TAG} > gpurun_out/pmc_${TAG}.txt 2>&1 || { tail -20 gpurun_out/pmc_${TAG}.txt; exit 1; }
  head -40 gpurun_out/pmc_${TAG}.txt
fi
