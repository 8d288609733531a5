#!/usr/bin/env bash
# A/B of an executor switch on one box: parity tests with the switch, then bench + per-layer
# kernel-time tables with and without it.
#   tools/gpu_ab_dw.sh <tag> <VAR=value> [pytest -k expr]
set -uo pipefail
TAG=${1:-ab}
SW=${2:-FSCNN_DW_DMA=1}
K=${3:-}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [[ -n "$K" ]]; then
  env $SW timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -k "$K" \
      > gpurun_out/ab_${TAG}_tests.log 2>&1
  rc=$?
  tail -3 gpurun_out/ab_${TAG}_tests.log
  [[ $rc -ne 0 ]] && { grep -E "^E |FAILED" gpurun_out/ab_${TAG}_tests.log | head -20; exit $rc; }
fi
for arm in base sw base sw; do
  if [[ $arm == sw ]]; then E="$SW"; else E="FSCNN_AB_BASE=1"; fi
  env $E timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extra --no-cfg5 --steps 20 \
      > gpurun_out/ab_${TAG}_${arm}.json 2> gpurun_out/ab_${TAG}_${arm}.err || { tail -20 gpurun_out/ab_${TAG}_${arm}.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_${TAG}_${arm}.json')); print('$arm', d['ms_per_step'], d['step_ms_distribution']['median'], d.get('forward_fp32',{}).get('ms_per_batch'), d.get('forward_fp32',{}).get('dw_fwd_hbm_frac'))"
done
for arm in base sw; do
  if [[ $arm == sw ]]; then E="$SW"; else E="FSCNN_AB_BASE=1"; fi
  OUT=gpurun_out/ab_${TAG}_layers_${arm}
  mkdir -p $OUT
  env $E timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- \
      python3 tools/rocprof_layers.py record $OUT/scopes.json > $OUT/record.log 2>&1 || { tail -20 $OUT/record.log; exit 1; }
  TR=$(find $OUT -name '*kernel_trace.csv' | head -1)
  python3 tools/rocprof_layers.py table "$TR" $OUT/scopes.json gpurun_out/ab_${TAG}_layers_${arm}.md > /dev/null || exit 1
  grep -A14 "kernel family" gpurun_out/ab_${TAG}_layers_${arm}.md | head -40
  rm -f "$TR"
done
