#!/usr/bin/env bash
# parity after the dw_wgrad workgroup-count change, then bench x2
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_fullsize.py tests/test_gpu_kernels.py tests/test_gpu_switches.py tests/test_gpu_train_api.py > gpurun_out/t20.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/t20.log | tail -8; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-forward --steps 30 > gpurun_out/b20.json 2> gpurun_out/b20.err || { tail -20 gpurun_out/b20.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/b20.json')); print(d['ms_per_step'], d['value'])"
done
