cd $GRAFT_REPO_ROOT
export STEM_DEBUG=1
timeout -k 10 120 python tests/_stem_worker.py gpurun_out/sd_a.npz && FSCNN_STEM_FUSED=0 timeout -k 10 120 python tests/_stem_worker.py gpurun_out/sd_b.npz && FSCNN_STEM_FUSED=0 timeout -k 10 120 python tests/_stem_worker.py gpurun_out/sd_c.npz && python3 - <<'PY'
import numpy as np
a, b, c = (dict(np.load("gpurun_out/sd_%s.npz" % k)) for k in "abc")
for k in sorted(a):
    if k == "stem_launches": continue
    print(k, "fused-vs-unfused", float(np.abs(a[k].astype(np.float64) - b[k]).max()), "unfused-vs-unfused", float(np.abs(c[k].astype(np.float64) - b[k]).max()))
PY
