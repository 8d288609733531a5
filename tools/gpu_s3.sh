#!/usr/bin/env bash
# low-M deep-K streaming GEMM: parity, predict fix, timing A/B, bench
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/diag_predict.py > gpurun_out/diag_predict.txt 2>&1 || { cat gpurun_out/diag_predict.txt; exit 1; }
cat gpurun_out/diag_predict.txt
timeout -k 10 600 python -u -m pytest -q -s --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "pw_gemm or bn_statistics" tests/test_gpu_switches.py::test_lowm_switch tests/test_gpu_fullsize.py -k "predict or pw_gemm or bn_statistics or lowm" > gpurun_out/t3.log 2>&1
rc=$?; grep -E "lowm vs|passed|failed|FAILED|Error" gpurun_out/t3.log | tail -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/lowres_gemm_bench.py > gpurun_out/gemm_lowm.txt 2>&1 || exit 1
FSCNN_GS_LOWM=0 timeout -k 10 120 python -u tools/lowres_gemm_bench.py > gpurun_out/gemm_tiled.txt 2>&1 || exit 1
paste gpurun_out/gemm_lowm.txt gpurun_out/gemm_tiled.txt | grep -v amdgpu.ids | cut -c1-200
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_s3.json 2> gpurun_out/bench_s3.err || { tail -20 gpurun_out/bench_s3.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_s3.json')); print(d['ms_per_step'], d['value'], d['roofline']['frac'], d['forward_fp32']['value'], d['forward_cfg5']['value'])"
