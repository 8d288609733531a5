#!/usr/bin/env bash
# Per-kernel VGPR / spill / occupancy / static LDS of one HIP source (gfx950).
#   tools/kres.sh <file.hip> [name-filter]
cd "$(dirname "$1")"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c "$(basename "$1")" -o /tmp/kres.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c "
import re, sys
flt = sys.argv[1] if len(sys.argv) > 1 else ''
cur = None
rows = []
for line in sys.stdin:
    m = re.search(r'remark:\s+(Function Name|VGPRs|VGPRs Spill|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\S+)', line)
    if not m:
        continue
    k, v = m.group(1), m.group(2)
    if k == 'Function Name':
        cur = {'name': v}
        rows.append(cur)
    else:
        cur[k] = v
for r in rows:
    if flt in r['name']:
        print('%-70s vgpr %4s spill %3s occ %s lds %s' % (r['name'][:70], r.get('VGPRs'), r.get('VGPRs Spill'), r.get('Occupancy [waves/SIMD]'), r.get('LDS Size [bytes/block]')))
" "${2:-}"
