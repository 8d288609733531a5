#!/usr/bin/env bash
# round-3 session check: GPU tests, bench line, host overhead
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gputests.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -5 gpurun_out/gputests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/bench_s1.json 2> gpurun_out/bench_s1.err || { tail -20 gpurun_out/bench_s1.err; exit 1; }
cat gpurun_out/bench_s1.json
timeout -k 10 120 python -u tools/host_overhead.py > gpurun_out/host_s1.txt 2>&1 || exit 1
tail -8 gpurun_out/host_s1.txt
