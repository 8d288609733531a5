#!/usr/bin/env bash
# CE head forms side by side: the 16-bit parity test and the stamped head launch per form.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for f in 1 2; do
  FSCNN_CE_HEAD=$f timeout -k 10 300 python -u -m pytest tests/test_gpu_literal.py -k ce_head_16bit -x -q \
      --timeout 120 --timeout-method thread > gpurun_out/ce_form$f.log 2>&1 || { tail -20 gpurun_out/ce_form$f.log; exit 1; }
  tail -1 gpurun_out/ce_form$f.log
  FSCNN_CE_HEAD=$f timeout -k 10 300 python -u tools/stamp_probe.py step > gpurun_out/ce_stamp$f.log 2>&1 || exit 1
  grep "head (upsample" gpurun_out/ce_stamp$f.log
done
