#!/usr/bin/env bash
# HBM traffic per dispatch of the bench train step, one rocprofv3 --pmc pass per counter group
# (never combined with runtime/sys traces).  MI355X_MICROARCH.md §HBM: FETCH_SIZE reads 1/2 of
# the bytes of 16-B/lane streaming reads on gfx950 (doubled by tools/pmc_summary.py);
# FETCH_SIZE and WRITE_SIZE do not fit one pass.
#   tools/pmc_step.sh <tag> [extra bench args]
set -euo pipefail
TAG=${1:-run}
shift || true
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/pmc_${TAG}
mkdir -p "$OUT"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"; do
  i=$((i + 1))
  timeout -k 10 400 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-forward --no-extra --profile-kind 3 "$@" \
      > "$OUT/p$i.log" 2>&1
  echo "pass $i ($grp) done"
done
python3 tools/pmc_summary.py "$OUT" --json-dir "$OUT" --tag "$TAG" --dtype bf16 > "$OUT/summary.txt"
cat "$OUT/summary.txt" | head -80
