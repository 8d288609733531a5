#!/usr/bin/env bash
# PMC HBM traffic with the side stream off (per-dispatch counters are unambiguous only when
# kernels do not overlap), then the dw_wgrad workgroup-count A/B
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out



bash tools/gpu_ab.sh "FSCNN_DWW_WG=1024" "FSCNN_DWW_WG=512" "FSCNN_DWW_WG=768"
