#!/usr/bin/env bash
# Kernel-level profile of the bench train step (and the fp32 forward) with rocprofv3.
#   tools/profile_step.sh <tag> [extra bench args]
# Writes gpurun_out/prof_<tag>/ (raw) and gpurun_out/prof_<tag>_kernel_stats.csv (summary).
set -euo pipefail
TAG=${1:-run}
shift || true
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/prof_${TAG}
mkdir -p "$OUT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra --profile-kind 3 --no-cfg5 "$@" > "$OUT/bench.log" 2>&1
STATS=$(find "$OUT" -name '*kernel_stats.csv' | head -1)
cp "$STATS" "gpurun_out/prof_${TAG}_kernel_stats.csv"
python3 - "$STATS" <<'EOF'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("kernel                                               calls   total_ms   avg_us   share")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:40]:
    print("%-52s %5s %10.3f %8.1f %6.1f%%" % (r["Name"][:52], r["Calls"], float(r["TotalDurationNs"]) / 1e6,
          float(r["AverageNs"]) / 1e3, 100 * float(r["TotalDurationNs"]) / tot))
print("total kernel ms: %.3f" % (tot / 1e6))
EOF
