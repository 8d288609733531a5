#!/usr/bin/env bash
# A/B/C... of executor switches on one box: bench (cfg3 train + cfg2 eval) per arm, twice,
# interleaved.   tools/gpu_ab_multi.sh <tag> <VAR=value> [<VAR=value> ...]   (arm "base" = none)
set -uo pipefail
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
  for SW in FSCNN_AB_BASE=1 "$@"; do
    name=${SW//[^A-Za-z0-9]/_}
    env $SW timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extra --no-cfg5 --steps 20 \
        > gpurun_out/ab_${TAG}_${name}_${rep}.json 2> gpurun_out/ab_${TAG}_${name}_${rep}.err || { tail -20 gpurun_out/ab_${TAG}_${name}_${rep}.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_${TAG}_${name}_${rep}.json')); print('$SW', d['ms_per_step'], d['step_ms_distribution']['median'], d.get('forward_fp32',{}).get('ms_per_batch'))"
  done
done
