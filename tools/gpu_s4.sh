#!/usr/bin/env bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/diag_predict.py low > gpurun_out/diag_low.txt 2>&1; cat gpurun_out/diag_low.txt | grep -v amdgpu.ids
timeout -k 10 400 python -u -m pytest -q -s --timeout 300 --timeout-method thread tests/test_gpu_switches.py::test_lowm_switch > gpurun_out/t4.log 2>&1
rc=$?; grep -E "lowm vs|passed|failed|FAILED|Error" gpurun_out/t4.log | tail -20; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python -u tools/lowres_gemm_bench.py > gpurun_out/gemm_lowm.txt 2>&1 || exit 1
FSCNN_GS_LOWM=0 timeout -k 10 120 python -u tools/lowres_gemm_bench.py > gpurun_out/gemm_tiled.txt 2>&1 || exit 1
paste -d'|' gpurun_out/gemm_lowm.txt gpurun_out/gemm_tiled.txt | grep -v amdgpu.ids | cut -c1-220
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_s4.json 2> gpurun_out/bench_s4.err || { tail -20 gpurun_out/bench_s4.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_s4.json')); print(d['ms_per_step'], d['value'], d['roofline']['frac'], d['forward_fp32']['value'], d['forward_cfg5']['value'])"
FSCNN_GS_LOWM=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-forward > gpurun_out/bench_s4t.json 2> gpurun_out/bench_s4t.err || { tail -20 gpurun_out/bench_s4t.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_s4t.json')); print('tiled', d['ms_per_step'], d['value'])"
