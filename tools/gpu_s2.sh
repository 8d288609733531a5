#!/usr/bin/env bash
# predict-vs-argmax diagnosis, then the whole GPU suite without -x
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/diag_predict.py > gpurun_out/diag_predict.txt 2>&1 || { cat gpurun_out/diag_predict.txt; exit 1; }
cat gpurun_out/diag_predict.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/gputests_all.log 2>&1
echo "tests rc=$?"
grep -E "passed|failed|FAILED|ERROR" gpurun_out/gputests_all.log | tail -20
