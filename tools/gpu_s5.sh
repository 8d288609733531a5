#!/usr/bin/env bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/diag_predict.py low > gpurun_out/diag_low.txt 2>&1; grep -v amdgpu.ids gpurun_out/diag_low.txt
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-forward > gpurun_out/bench_s5.json 2> gpurun_out/bench_s5.err || { tail -20 gpurun_out/bench_s5.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_s5.json')); print(d['ms_per_step'], d['value'], d['roofline']['frac'])"
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-forward > gpurun_out/bench_s5b.json 2> gpurun_out/bench_s5b.err || { tail -20 gpurun_out/bench_s5b.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_s5b.json')); print(d['ms_per_step'], d['value'], d['roofline']['frac'])"
