#!/usr/bin/env bash
# stride-2 dgrad parity + per-layer table, then the low-res GEMM microbenchmark under rocprofv3
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_dwtest.sh || exit 1
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/lowres_gemm_bench.py > gpurun_out/gemm_bench.log 2>&1 || exit 1
cat gpurun_out/gemm_bench.log
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gemm -o gb -- python3 tools/lowres_gemm_bench.py --reps 20 > gpurun_out/gemm_prof.log 2>&1 || exit 1
find gpurun_out/prof_gemm -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/gemm_kernel_stats.csv
