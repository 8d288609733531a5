set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/abup; mkdir -p $O
timeout -k 10 180 python -u tools/ffm_bitcheck.py 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_dsconv.py "tests/test_gpu_switches.py::test_ffm_hi_fused_bit_identical" "tests/test_gpu_switches.py::test_dsconv_fused_bit_identical" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
for rep in 1 2; do
  for lib in abl/old.so fast-scnn-pytorch_amd/libfastscnn_hip.so; do
    FSCNN_LIB=$lib timeout -k 10 120 python tools/fwd_run.py --cfg 2 --reps 30 2>&1 | tail -n 1 | sed "s|^|$lib |" || exit 1
    FSCNN_LIB=$lib timeout -k 10 120 python tools/fwd_run.py --cfg 5 --reps 30 2>&1 | tail -n 1 | sed "s|^|$lib |" || exit 1
  done
done
