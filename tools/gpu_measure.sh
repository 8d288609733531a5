#!/usr/bin/env bash
# Round measurement set: full GPU suite, smoke, the bench line, rocprofv3 kernel stats + one
# train step trace, the family kernel times the bench reads, PMC HBM traffic, per-layer tables.
#   tools/gpu_measure.sh <tag>
set -uo pipefail
TAG=${1:-r06}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
O=gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/gputests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED|ERROR" $O/gputests.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash tools/profile_step.sh $TAG --no-forward > $O/prof.txt 2>&1 || { tail -20 $O/prof.txt; exit 1; }
head -30 $O/prof.txt
TR=$(find gpurun_out/prof_$TAG -name '*kernel_trace.csv' | head -1)
python3 tools/trace_step.py "$TR" --step 4 > $O/train_step_trace.txt || exit 1
rm -f "$TR"
python3 tools/rocprof_family.py gpurun_out/prof_${TAG}_kernel_stats.csv $TAG $O/rocprof_family_bf16.json || exit 1
FSCNN_SIDE_STREAM=0 bash tools/pmc_step.sh $TAG > $O/pmc.txt 2>&1 || { tail -20 $O/pmc.txt; exit 1; }
head -20 $O/pmc.txt
mkdir -p $O/layers
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/layers/tr -o run -- \
    python3 tools/rocprof_layers.py record $O/layers/scopes.json > $O/layers/rec.log 2>&1 || { tail -20 $O/layers/rec.log; exit 1; }
LT=$(find $O/layers/tr -name '*kernel_trace.csv' | head -1)
python3 tools/rocprof_layers.py table "$LT" $O/layers/scopes.json $O/layers.md > /dev/null || exit 1
rm -f "$LT"
grep -A16 "kernel family" $O/layers.md | head -40
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
