#!/usr/bin/env bash
# worst gradient-gate ratios of the fp32 oracle tests under executor switches
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for combo in "$@"; do
  env $combo timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -q -s -k "train_fp32_streaming" \
      --timeout 200 --timeout-method thread > gpurun_out/ratio.log 2>&1
  rc=$?
  echo "== $combo: $(tail -1 gpurun_out/ratio.log)"
  grep "grad gate" gpurun_out/ratio.log
  if [[ $rc -ne 0 && $rc -ne 1 ]]; then exit $rc; fi
done
