"""Where k_resolve spills: compile ie_resolve.hip to device asm and list, per instance, the
source lines (from the asm's .loc directives) nearest to each scratch store / load."""
import collections
import re
import subprocess
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "ie_resolve.hip"
want = sys.argv[2] if len(sys.argv) > 2 else "Lb0ELb0ELb0E"
subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-g",
                       "-mllvm", "-amdgpu-sched-strategy=max-ilp", "-S", "--offload-device-only", src,
                       "-o", "/tmp/spills.s"], cwd="interpolation-engine_amd/csrc", stderr=subprocess.DEVNULL)
s = open("/tmp/spills.s").read()
files = dict(re.findall(r'\.file\s+(\d+)\s+"[^"]*"\s+"([^"]+)"', s))
for f in re.split(r"\n(?=_ZN2ie4r2569k_resolveI\w+:)", s):
    m = re.match(r"_ZN2ie4r2569k_resolveI(\w+)EEvNS\w+:", f)
    if not m or m.group(1) != want:
        continue
    loc = "?"
    c = collections.Counter()
    for line in f.split("\n"):
        mm = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", line)
        if mm:
            loc = "%s:%s" % (files.get(mm.group(1), mm.group(1)).split("/")[-1], mm.group(2))
        if "scratch_store" in line or "scratch_load" in line:
            c[("st " if "store" in line else "ld ") + loc] += 1
    for k, v in sorted(c.items(), key=lambda kv: -kv[1])[:25]:
        print(v, k)
