#!/usr/bin/env bash
# One GPU session (round 3): bench line, rocprofv3 kernel stats of the train step, and the
# printed parity figures (fp16 / bf16 AMP budgets, argmax flip counts, DataParallel grads).
#   tools/gpu_r03.sh <tag> [bench|prof|prints|all]...
set -uo pipefail
TAG=${1:-run}
shift || true
WHAT=${*:-all}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
has() { [[ " $WHAT " == *" $1 "* || " $WHAT " == *" all "* ]]; }
if has bench; then
  timeout -k 10 500 python -u bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err \
    || { tail -20 gpurun_out/bench_${TAG}.err; exit 1; }
  cat gpurun_out/bench_${TAG}.json
fi
if has prints; then
  timeout -k 10 400 python -u -m pytest -q -s --timeout 300 --timeout-method thread \
      tests/test_gpu_fullsize.py tests/test_gpu_train_api.py::test_autocast_gradscaler_step_as_train_py \
      tests/test_gpu_dataparallel.py -k "literal or goldens or budget or autocast or replicate" \
      > gpurun_out/prints_${TAG}.log 2>&1 || { tail -30 gpurun_out/prints_${TAG}.log; exit 1; }
  grep -E "argmax:|train step:|fp16 AMP|worst relative|cfg5 fp16|passed|failed" gpurun_out/prints_${TAG}.log
fi
if has prof; then
  bash tools/profile_step.sh ${TAG} --no-forward > gpurun_out/prof_${TAG}.txt 2>&1 \
    || { tail -20 gpurun_out/prof_${TAG}.txt; exit 1; }
  head -30 gpurun_out/prof_${TAG}.txt
fi
