#!/usr/bin/env bash
# A/B of environment knobs on the bench train step: tools/gpu_ab.sh "ENV=V ..." ...
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for rep in 1 2; do
for cfg in "$@"; do
  env $cfg timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-forward --no-extra --steps 30 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab.json')); print(sys.argv[1], d['ms_per_step'], d['value'])" "$cfg"
done
done
