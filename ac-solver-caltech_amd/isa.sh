#!/bin/bash
# Dump gfx950 ISA of the L=36 kernels for inspection: isa.sh [outdir]
set -e
D=$(cd "$(dirname "$0")" && pwd)
OUT=${1:-/tmp/isa}
mkdir -p $OUT
hipcc --offload-arch=gfx950 -O3 -std=c++17 -I$D/../include --cuda-device-only -S -DACX_ISA_L36_ONLY \
  -Wno-pass-failed -o $OUT/acx36.s $D/csrc/acx_kernels.hip 2>&1 | grep -v hip-link || true
python3 - "$OUT" <<'PY'
import re, sys
out = sys.argv[1]
s = open(out + '/acx36.s').read()
for k in re.findall(r'^(_ZN3acx\w+):', s, re.M):
    if '.name:           ' + k not in s:  # an out-of-line device function, not a kernel
        continue
    i = s.index(k + ':'); j = s.index('.Lfunc_end', i)
    short = re.sub(r'_ZN3acx\d+(\w+?)_kernel.*', r'\1', k)
    open(f'{out}/{short}.s', 'w').write(s[i:j])
    m = s.index('.name:           ' + k)
    v = re.findall(r'\.vgpr_count:\s+(\d+)', s[m:m + 3000])[0]
    g = re.findall(r'\.sgpr_count:\s+(\d+)', s[m:m + 3000])[0]
    n = sum(1 for l in s[i:j].split('\n') if l.startswith('\t') and not l.startswith('\t.') and not l.startswith('\t;'))
    print(f'{short:10s} vgpr {v:>4} sgpr {g:>4} instructions {n}')
PY
