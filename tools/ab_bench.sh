#!/usr/bin/env bash
# A/B the bench train step AND the cfg2 fp32 forward over executor switches:
#   tools/ab_bench.sh <tag> "ENV=.. ENV=.." ...
set -uo pipefail
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for combo in "$@"; do
  env $combo timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-cfg5 --steps 30 \
      > gpurun_out/ab_${TAG}.json 2> gpurun_out/ab_${TAG}.err || { tail -5 gpurun_out/ab_${TAG}.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_${TAG}.json')); print('%-40s %.3f ms/step  fwd fp32 %.3f ms/batch' % (sys.argv[1], d['ms_per_step'], d['forward_fp32']['ms_per_batch']))" "$combo"
done
