#!/usr/bin/env bash
# One rocprofv3 --pmc pass of SQ counters over the bench train step (2 steps), summarised for the
# kernels whose name matches a pattern: where a kernel's wave cycles go (VALU issue vs waits).
#   tools/pmc_sq.sh <tag> <kernel-substring> [counters...]
# PMC_EVAL=<cfg>: profile tools/fwd_run.py's eval forward of that config instead of the train step.
set -euo pipefail
TAG=${1:-run}; PAT=${2:-ce_head}; shift 2 || true
CTRS=${*:-"SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS"}
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/pmcsq_${TAG}
mkdir -p "$OUT"
if [ -n "${PMC_EVAL:-}" ]; then
  timeout -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv -d "$OUT/p" -o run -- \
      python3 tools/fwd_run.py --cfg "$PMC_EVAL" --reps 2 > "$OUT/p.log" 2>&1
else
  timeout -s KILL 300 rocprofv3 --pmc $CTRS --output-format csv -d "$OUT/p" -o run -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-forward --no-extra > "$OUT/p.log" 2>&1
fi
python3 - "$OUT" "$PAT" <<'PY'
import csv, glob, os, sys, collections
out, pat = sys.argv[1], sys.argv[2]
rows = []
for f in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
    rows += list(csv.DictReader(open(f)))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for r in rows:
    if pat in r["Kernel_Name"]:
        k = r["Kernel_Name"][:70]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        n[(k, r["Counter_Name"])] += 1
for k, c in agg.items():
    print(k)
    for name, v in sorted(c.items()):
        print("  %-24s %16.0f  (dispatches %d)" % (name, v, n[(k, name)]))
PY
