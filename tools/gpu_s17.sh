#!/usr/bin/env bash
# fused LTD.dsconv1.dw dgrad + conv0 wgrad: parity (fused vs two-pass, bf16 budget), then A/B
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread "tests/test_gpu_switches.py::test_ltd_fused_backward_matches_two_pass" > gpurun_out/t17a.log 2>&1
rc=$?; tail -30 gpurun_out/t17a.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fullsize.py tests/test_gpu_model.py > gpurun_out/t17b.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/t17b.log | tail -8; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab.sh "FSCNN_LTD_FUSED=0" "FSCNN_LTD_FUSED=1"
