#!/usr/bin/env bash
# One GPU session: gpu tests, bench (default and without lazy BN), eval forward, kernel profile.
#   tools/gpu_round.sh <tag>
set -euo pipefail
TAG=${1:-run}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/gputest_${TAG}.log 2>&1 || { tail -30 gpurun_out/gputest_${TAG}.log; exit 1; }
tail -3 gpurun_out/gputest_${TAG}.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err
cat gpurun_out/bench_${TAG}.json
FSCNN_LAZY_BN=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-forward \
    > gpurun_out/bench_${TAG}_nolazy.json 2>> gpurun_out/bench_${TAG}.err
python3 -c "import json;d=json.load(open('gpurun_out/bench_${TAG}_nolazy.json'));print('nolazy', d['ms_per_step'], d['value'])"
timeout -k 10 200 python -u tools/fwd_run.py --cfg 2 --reps 20
bash tools/profile_step.sh ${TAG} > gpurun_out/prof_${TAG}.txt 2>&1
head -45 gpurun_out/prof_${TAG}.txt
