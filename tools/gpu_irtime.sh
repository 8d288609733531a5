#!/usr/bin/env bash
# fused inference bottleneck: parity vs torch, then the per-layer eval table (fused rows)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 python -u -m pytest -q -s --timeout 120 --timeout-method thread tests/test_gpu_ir_block.py > gpurun_out/ir.log 2>&1; tail -4 gpurun_out/ir.log
timeout -k 10 300 python -u tools/layer_report.py gpurun_out/layers_ir.md > gpurun_out/lr.log 2>&1
grep -A 40 "cfg2 eval" gpurun_out/layers_ir.md | grep -E "fused|Total|ir_block"
