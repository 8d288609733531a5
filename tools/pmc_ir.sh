#!/usr/bin/env bash
# PMC counters of the fused inference bottleneck kernel (one rocprofv3 --pmc pass per group)
set -uo pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/pmc_ir
mkdir -p $OUT
for dt in fp32 bf16; do timeout -k 10 60 python3 tools/ir_bench.py --dtype $dt; done
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_VALU_MFMA_BUSY_CYCLES"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- \
      python3 tools/ir_bench.py --reps 3 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; }
  f=$(find $OUT/p$i -name '*counter_collection.csv' | head -1)
  [ -n "$f" ] && python3 - "$f" <<'PY'
import csv, sys, collections
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "ir_block" in r.get("Kernel_Name", "")]
acc = collections.defaultdict(float)
for r in rows:
    acc[r["Counter_Name"]] += float(r["Counter_Value"])
n = max(1, len({r["Dispatch_Id"] for r in rows}))
for k, v in sorted(acc.items()):
    print("%-28s %.4g per dispatch" % (k, v / n))
PY
done
