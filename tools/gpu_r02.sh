#!/usr/bin/env bash
# One GPU session (round 2): gpu tests, bench, train-step kernel profile (train only), smoke.
#   tools/gpu_r02.sh <tag> [tests|bench|prof|all]
set -uo pipefail
TAG=${1:-run}
WHAT=${2:-all}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
if [[ $WHAT == all || $WHAT == tests ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread \
      -rA > gpurun_out/gputest_${TAG}.log 2>&1
  rc=$?
  grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/gputest_${TAG}.log | tail -60
  if [[ $rc -ne 0 && $rc -ne 1 ]]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
fi
if [[ $WHAT == all || $WHAT == bench ]]; then
  timeout -k 10 500 python -u bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { tail -20 gpurun_out/bench_${TAG}.err; exit 1; }
  cat gpurun_out/bench_${TAG}.json
fi
if [[ $WHAT == all || $WHAT == prof ]]; then
  bash tools/profile_step.sh ${TAG} --no-forward > gpurun_out/prof_${TAG}.txt 2>&1 || { tail -20 gpurun_out/prof_${TAG}.txt; exit 1; }
  head -60 gpurun_out/prof_${TAG}.txt
fi
