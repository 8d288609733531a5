set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/ffm; mkdir -p $O
timeout -k 10 180 python -u tools/ffm_bitcheck.py 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_dsconv.py "tests/test_gpu_switches.py::test_ffm_hi_fused_bit_identical" "tests/test_gpu_switches.py::test_dsconv_fused_bit_identical" "tests/test_gpu_switches.py::test_switch_keeps_oracle_parity[FSCNN_FFM_HI=0]" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
