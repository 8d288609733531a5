#!/usr/bin/env bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_fullsize.py tests/test_gpu_train_api.py > gpurun_out/t15.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/t15.log | tail -8; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-forward --steps 30 > gpurun_out/bench_s15.json 2> gpurun_out/bench_s15.err || { tail -20 gpurun_out/bench_s15.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_s15.json')); c=d['kernel_ms_per_step_census']; print(d['ms_per_step'], d['value'], c['ppm_branches'])"
done
bash tools/profile_step.sh r03c --no-forward > gpurun_out/prof_r03c.txt 2>&1 || exit 1
grep -E "ppm|pyramid|pool" gpurun_out/prof_r03c.txt
