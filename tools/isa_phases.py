"""Static instruction counts of one k_resolve instance between consecutive s_memrealtime
instructions (the IE_STAMP / resolve_jobs stamp markers), in program order: a rough map of how
much code each phase is (loops counted once). Usage: python tools/isa_phases.py [asm] [suffix]"""
import collections
import re
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "/tmp/isa.s"
suffix = sys.argv[2] if len(sys.argv) > 2 else "Lb0ELb0ELb1ELb0ELb0E"
s = open(path).read()
name = "_ZN2ie4r2569k_resolveI%sEEvNS_5BatchENS_4WorkENS_8DevTableEPhm" % suffix
a = s.index("\n" + name + ":")
b = s.index("s_endpgm", a)
segs, cur, locs = [], collections.Counter(), collections.Counter()
for line in s[a:b].split("\n")[1:]:
    t = line.strip()
    m = re.match(r"\.loc\s+\d+\s+(\d+)", t)
    if m:
        locs[int(m.group(1))] += 1
        continue
    if not t or t.startswith((".", ";")) or t.endswith(":"):
        continue
    op = t.split()[0]
    cls = "valu" if op.startswith("v_") else "salu" if op.startswith("s_") else "lds" if op.startswith("ds_") \
        else "vmem" if op.startswith(("global_", "buffer_", "flat_", "scratch_")) else "other"
    cur[cls] += 1
    if op == "s_memrealtime":
        segs.append(dict(cur))
        cur = collections.Counter()
segs.append(dict(cur))
for k, c in enumerate(segs):
    print(k, c)
