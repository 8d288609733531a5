#!/usr/bin/env bash
# One GPU session (round 4).  Steps run in order, each under its own time limit, and the script
# stops at the first failure.
#   tools/gpu_r04.sh <tag> step...
#   steps: tests[=pytest -k expr] | bench | quick (bench, train only) | prof | smoke | file:<path.py>
set -uo pipefail
TAG=${1:-run}
shift || true
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for step in "$@"; do
  case "$step" in
    tests)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
          > gpurun_out/tests_${TAG}.log 2>&1
      rc=$?; grep -E "passed|failed|FAILED|ERROR" gpurun_out/tests_${TAG}.log | tail -8
      [ $rc -eq 0 ] || exit $rc ;;
    tests=*)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
          -k "${step#tests=}" > gpurun_out/tests_${TAG}.log 2>&1
      rc=$?; grep -E "PASSED|passed|failed|FAILED|ERROR" gpurun_out/tests_${TAG}.log | tail -30
      [ $rc -eq 0 ] || exit $rc ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1 \
          || { tail -5 gpurun_out/smoke_${TAG}.log; exit 1; }
      tail -1 gpurun_out/smoke_${TAG}.log ;;
    bench)
      timeout -k 10 600 python -u bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err \
          || { tail -20 gpurun_out/bench_${TAG}.err; exit 1; }
      cat gpurun_out/bench_${TAG}.json ;;
    quick)
      timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-forward --no-extra > gpurun_out/quick_${TAG}.json \
          2> gpurun_out/quick_${TAG}.err || { tail -20 gpurun_out/quick_${TAG}.err; exit 1; }
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ms_per_step'], d['value'], d['roofline'])" \
          gpurun_out/quick_${TAG}.json ;;
    prof)
      bash tools/profile_step.sh ${TAG} --no-forward > gpurun_out/prof_${TAG}.txt 2>&1 \
          || { tail -20 gpurun_out/prof_${TAG}.txt; exit 1; }
      head -45 gpurun_out/prof_${TAG}.txt ;;
    ab=*)  # ab=A=1+B=2,A=0 : configs separated by ',', env vars of one config by '+'
      IFS=',' read -ra cfgs <<< "${step#ab=}"
      args=()
      for c in "${cfgs[@]}"; do args+=("${c//+/ }"); done
      bash tools/gpu_ab.sh "${args[@]}" || exit 1 ;;
    file:*)
      f=${step#file:}
      timeout -k 10 400 python -u $f > gpurun_out/$(basename $f .py)_${TAG}.log 2>&1
      rc=$?; tail -40 gpurun_out/$(basename $f .py)_${TAG}.log
      [ $rc -eq 0 ] || exit $rc ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
