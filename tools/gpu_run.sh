#!/usr/bin/env bash
# GPU iteration: selected GPU tests, then the bench train step + cfg2 forward (no CPU baseline).
#   tools/gpu_run.sh <tag> [pytest args, e.g. tests/test_gpu_bf16_train.py -k expr]
set -uo pipefail
TAG=${1:-q}; shift || true
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [[ $# -gt 0 ]]; then
  timeout -k 10 900 python -u -m pytest -m gpu -x -v -s --timeout 300 --timeout-method thread "$@" \
      > gpurun_out/t_${TAG}.log 2>&1
  rc=$?
  grep -E "PASSED|FAILED|ERROR|passed|failed|cosine|ratio|flips|loss:" gpurun_out/t_${TAG}.log | tail -40
  [[ $rc -eq 0 ]] || { echo "pytest rc=$rc: stopping"; exit $rc; }
fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extra --no-cfg5 \
    > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { tail -20 gpurun_out/bench_${TAG}.err; exit 1; }
python3 - gpurun_out/bench_${TAG}.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r = d["roofline"]
print("ms/step %.3f median %.3f  value %.1f  roofline %s %.4f (avg %.2f us, rocprof %s)" % (
    d["ms_per_step"], d["step_ms_distribution"]["median"], d["value"], r["kernel"], r["frac"],
    r["avg_launch_us"], r.get("rocprof", {}).get("frac")))
for k, v in d.get("depthwise_train", {}).items():
    if k != "note":
        print("  %-9s %3d launches %8.1f us  frac %.3f" % (k, v["launches"], v["us"], v["hbm_frac"]))
f = d.get("forward_fp32", {})
print("fwd fp32 %.3f ms/batch" % f.get("ms_per_batch", 0), json.dumps(f.get("fused_blocks_mfma")))
PY
