#!/usr/bin/env bash
# Quick GPU iteration: model parity tests, bench (no CPU baseline), train-step profile.
#   tools/gpu_quick.sh <tag> [pytest -k expr]
set -uo pipefail
TAG=${1:-q}
K=${2:-}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
if [[ -n "$K" ]]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -k "$K" \
      > gpurun_out/gputest_${TAG}.log 2>&1
else
  timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_kernels.py -m gpu -q \
      --timeout 200 --timeout-method thread > gpurun_out/gputest_${TAG}.log 2>&1
fi
rc=$?
tail -5 gpurun_out/gputest_${TAG}.log
if [[ $rc -ne 0 && $rc -ne 1 ]]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-cfg5 > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { tail -20 gpurun_out/bench_${TAG}.err; exit 1; }
cat gpurun_out/bench_${TAG}.json
bash tools/profile_step.sh ${TAG} --no-forward > gpurun_out/prof_${TAG}.txt 2>&1 || { tail -20 gpurun_out/prof_${TAG}.txt; exit 1; }
python3 tools/prof_table.py gpurun_out/prof_${TAG}_kernel_stats.csv 7 40
