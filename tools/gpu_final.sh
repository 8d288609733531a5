#!/usr/bin/env bash
# round-3 final measurement: full GPU suite, smoke, full bench line, profile set with PMC
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/gputests_final.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED|ERROR" gpurun_out/gputests_final.log | tail -5
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 || { tail -5 gpurun_out/smoke_final.log; exit 1; }
tail -1 gpurun_out/smoke_final.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { tail -20 gpurun_out/bench_final.err; exit 1; }
cat gpurun_out/bench_final.json
bash tools/gpu_prof.sh r03i pmc
