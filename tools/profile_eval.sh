#!/usr/bin/env bash
# Kernel profile of the eval forward (cfg2 fp32, and cfg5 fp16 I/O) with rocprofv3.
#   tools/profile_eval.sh <tag>
set -euo pipefail
TAG=${1:-run}
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for CFG in 2 5; do
  OUT=gpurun_out/prof_${TAG}_eval${CFG}
  mkdir -p "$OUT"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
      python3 tools/fwd_run.py --cfg $CFG --reps 10 > "$OUT/run.log" 2>&1
  cat "$OUT/run.log" | grep forward
  STATS=$(find "$OUT" -name '*kernel_stats.csv' | head -1)
  cp "$STATS" "gpurun_out/prof_${TAG}_eval${CFG}_kernel_stats.csv"
  python3 tools/prof_table.py "gpurun_out/prof_${TAG}_eval${CFG}_kernel_stats.csv" 13 25
done
