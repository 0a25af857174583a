#!/bin/bash
# Per-kernel VGPRs / scratch / occupancy of kernels.hip (compile-only; filter by regex $1)
cd "$(dirname "$0")/../pinot_amd/csrc"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -I../../include --offload-arch=gfx950 -munsafe-fp-atomics -ffp-contract=off \
  -c kernels.hip -Rpass-analysis=kernel-resource-usage -o /tmp/res.o 2>&1 | python3 -c "
import re,sys
cur=None; rows={}
for l in sys.stdin:
    m=re.search(r'Function Name: (\S+)',l)
    if m: cur=m.group(1); rows[cur]={}; continue
    m=re.search(r'remark:\s+([A-Za-z ]+?)(?: \[[^]]*\])?: (\d+)',l)
    if m and cur: rows[cur][m.group(1).strip()]=m.group(2)
pat=re.compile(sys.argv[1] if len(sys.argv)>1 else '.')
for f,r in rows.items():
    if pat.search(f): print(f[:48].ljust(48), 'vgpr',r.get('VGPRs'),'scratch',r.get('ScratchSize'),'occ',r.get('Occupancy'),'sgpr_spill',r.get('SGPRs Spill'))
" "${1:-.}"
