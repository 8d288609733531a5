#!/usr/bin/env bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/gputests_s8.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED|ERROR" gpurun_out/gputests_s8.log | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/gpu_prof.sh r03a
