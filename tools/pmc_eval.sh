#!/usr/bin/env bash
# HBM traffic and issue counters per dispatch of the eval forward (cfg2 fp32 by default), one
# rocprofv3 --pmc pass per counter group (never combined with runtime/sys traces), summarised per
# kernel: FETCH_SIZE / WRITE_SIZE in KB per dispatch (FETCH_SIZE x 2 = the gfx950 correction for
# 16-B/lane streaming reads, MI355X_MICROARCH.md), MFMA busy and VALU instructions per dispatch.
#   tools/pmc_eval.sh <tag> [cfg]
set -euo pipefail
TAG=${1:-run}
CFG=${2:-2}
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/pmce_${TAG}
mkdir -p "$OUT"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- \
      python3 tools/fwd_run.py --cfg "$CFG" --reps 2 > "$OUT/p$i.log" 2>&1
  echo "pass $i ($grp) done"
done
python3 - "$OUT" <<'PY' | tee "$OUT/summary.txt"
import csv, glob, os, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(lambda: collections.Counter())
for f in glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][:64]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[k][r["Counter_Name"]] += 1
print("%-64s %9s %9s %9s %7s %9s" % ("kernel", "fetchKBx2", "writeKB", "mfma_us", "waves", "valu_k"))
rows = []
for k, c in agg.items():
    n = lambda name: max(1, cnt[k][name])  # noqa: E731
    fetch = 2 * c.get("FETCH_SIZE", 0) / n("FETCH_SIZE")
    write = c.get("WRITE_SIZE", 0) / n("WRITE_SIZE")
    mfma = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / n("SQ_VALU_MFMA_BUSY_CYCLES") / 2.4e3 / 1024
    waves = c.get("SQ_WAVES", 0) / n("SQ_WAVES")
    valu = c.get("SQ_INSTS_VALU", 0) / n("SQ_INSTS_VALU") / 1e3
    rows.append((fetch + write, k, fetch, write, mfma, waves, valu))
for _, k, fetch, write, mfma, waves, valu in sorted(rows, reverse=True)[:30]:
    print("%-64s %9.0f %9.0f %9.1f %7.0f %9.0f" % (k, fetch, write, mfma, waves, valu))
print("(mfma_us: SQ_VALU_MFMA_BUSY_CYCLES per dispatch / 2.4 GHz / 1024 SIMDs = the kernel time its"
      " MFMA work would take at the dense peak)")
PY
