#!/usr/bin/env bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_fullsize.py tests/test_gpu_train_api.py tests/test_gpu_switches.py tests/test_gpu_dataparallel.py tests/test_gpu_ddp.py > gpurun_out/t16.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/t16.log | tail -8; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-forward --steps 30 > gpurun_out/bench_s16.json 2> gpurun_out/bench_s16.err || { tail -20 gpurun_out/bench_s16.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_s16.json')); print(d['ms_per_step'], d['value'])"
done
