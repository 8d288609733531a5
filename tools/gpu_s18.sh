#!/usr/bin/env bash
# CE head (tree reductions, v_log_f32) + ltd 32-bit tile math: parity then bench x3
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_fullsize.py "tests/test_gpu_switches.py::test_ltd_fused_backward_matches_two_pass" > gpurun_out/t18.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/t18.log | tail -8; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-forward --steps 30 > gpurun_out/b18.json 2> gpurun_out/b18.err || { tail -20 gpurun_out/b18.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/b18.json')); print(d['ms_per_step'], d['value'])"
done
