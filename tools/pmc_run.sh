#!/usr/bin/env bash
# PMC counters per dispatch for any python command, one rocprofv3 --pmc pass per counter group
# (never combined with runtime/sys traces; MI355X_MICROARCH.md §HBM).  FETCH_SIZE and WRITE_SIZE
# do not fit one pass.
#   tools/pmc_run.sh <tag> <python args...>      e.g. tools/pmc_run.sh fwd2 tools/fwd_run.py --reps 2
set -euo pipefail
TAG=$1
shift
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/pmc_${TAG}
mkdir -p "$OUT"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU"; do
  i=$((i + 1))
  timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- python3 "$@" \
      > "$OUT/p$i.log" 2>&1
  echo "pass $i ($grp) done"
done
