#!/bin/bash
# Where the LEAN k_resolve instance spills (-DIE_EXP_ONLY_LEAN compile; extra hipcc flags as args):
# scratch stores / loads per source line (the asm's .loc directives)
cd "$(dirname "$0")/../interpolation-engine_amd/csrc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -g -mllvm -amdgpu-sched-strategy=max-ilp \
  -DIE_EXP_ONLY_LEAN "$@" -S --offload-device-only ie_resolve.hip -o /tmp/lean_spills.s 2>/dev/null
python3 - <<'PY'
import re, collections
s = open('/tmp/lean_spills.s').read()
files = dict(re.findall(r'\.file\s+(\d+)\s+"[^"]*"\s+"([^"]+)"', s))
for f in re.split(r"\n(?=_ZN2ie4r2569k_resolveI\w+:)", s):
    m = re.match(r"_ZN2ie4r2569k_resolveI(\w+)EEvNS\w+:", f)
    if not m or m.group(1) != 'Lb0ELb0ELb1ELb0ELb0ELb1E':
        continue
    loc = '?'; c = collections.Counter()
    for line in f.split('\n'):
        mm = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", line)
        if mm:
            loc = "%s:%s" % (files.get(mm.group(1), mm.group(1)).split('/')[-1], mm.group(2))
        if 'scratch_store' in line or 'scratch_load' in line:
            c[('st ' if 'store' in line else 'ld ') + loc] += 1
    for k, v in sorted(c.items(), key=lambda kv: -kv[1])[:30]:
        print(v, k)
PY
