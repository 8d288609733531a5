#!/usr/bin/env bash
# fp32 gradient parity per in-kernel BN finish producer (FSCNN_TAIL_INK bitmask)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for m in 1 2 4 8; do
  FSCNN_TAIL_INK=$m timeout -k 10 200 python -u -m pytest tests/test_gpu_model.py -x -q -k "train_fp32" \
      --timeout 200 --timeout-method thread > gpurun_out/t_bis$m.log 2>&1
  rc=$?
  echo "mask $m: $(tail -1 gpurun_out/t_bis$m.log)"
  if [[ $rc -ne 0 && $rc -ne 1 ]]; then exit $rc; fi
done
