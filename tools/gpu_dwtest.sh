#!/usr/bin/env bash
# depthwise kernel parity + train-step parity, then the per-layer train table (dw_dgrad rows)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_fullsize.py -k "dw or train or budget" > gpurun_out/dwt.log 2>&1; tail -3 gpurun_out/dwt.log
grep -E "FAIL|Error" gpurun_out/dwt.log | head -10
FSCNN_SIDE_STREAM=0 timeout -k 10 300 python -u tools/layer_report.py gpurun_out/dw_layers.md > gpurun_out/dwl.log 2>&1
grep -E "dw_dgrad|^\| dw_|gemm_nt \||Total over" gpurun_out/dw_layers.md | head -30
