#!/usr/bin/env bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_fullsize.py tests/test_gpu_kernels.py -k "predict or pw_gemm or bn_statistics or bilinear or argmax" > gpurun_out/t7.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/t7.log | tail -8; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for t in 1024 512 256 1024 512 256; do
  FSCNN_TN_WG=$t timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-forward --steps 30 > gpurun_out/bench_tn$t.json 2> gpurun_out/bench_tn$t.err || { tail -20 gpurun_out/bench_tn$t.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/bench_tn$t.json')); print('tn target $t', d['ms_per_step'], d['value'], d['kernel_ms_per_step_census']['gemm_tn'])"
done
