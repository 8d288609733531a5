#!/usr/bin/env bash
# Per-layer kernel-time table (rocprofv3 kernel trace, side stream off): tools/rocprof_layers.py
#   tools/gpu_layers.sh <tag> [ENV=value ...]
set -uo pipefail
TAG=${1:-l}; shift || true
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/layers_$TAG
mkdir -p $O
env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- \
    python3 tools/rocprof_layers.py record $O/scopes.json > $O/rec.log 2>&1 || { tail -20 $O/rec.log; exit 1; }
LT=$(find $O/tr -name '*kernel_trace.csv' | head -1)
python3 tools/rocprof_layers.py table "$LT" $O/scopes.json $O/layers.md > /dev/null || exit 1
rm -f "$LT"
grep -A18 "kernel family" $O/layers.md | head -20
