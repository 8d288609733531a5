#!/usr/bin/env bash
# A/B the bench step time over executor switches: tools/ab_env.sh <tag> "ENV=.. ENV=.." ...
set -uo pipefail
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for combo in "$@"; do
  env $combo timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-cfg5 --steps 30 \
      > gpurun_out/ab_${TAG}.json 2> gpurun_out/ab_${TAG}.err || { tail -5 gpurun_out/ab_${TAG}.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_${TAG}.json')); print('%-45s %.3f ms/step' % (sys.argv[1], d['ms_per_step']))" "$combo"
done
