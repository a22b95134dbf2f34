"""Static VALU / SALU / LDS / VMEM instruction counts of one k_resolve instance, attributed to the
source line of each instruction (the asm's .loc directives), grouped by function-sized line ranges
of ie_resolve.hip. A map of where the code is, not a dynamic count (loops are counted once)."""
import collections
import re
import subprocess
import sys

want = sys.argv[1] if len(sys.argv) > 1 else "Lb0ELb0ELb1E"
subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-g",
                       "-mllvm", "-amdgpu-sched-strategy=max-ilp", "-S", "--offload-device-only", "ie_resolve.hip",
                       "-o", "/tmp/isa.s"], cwd="interpolation-engine_amd/csrc", stderr=subprocess.DEVNULL)
s = open("/tmp/isa.s").read()
files = dict(re.findall(r'\.file\s+(\d+)\s+"[^"]*"\s+"([^"]+)"', s))
src = open("interpolation-engine_amd/csrc/ie_resolve.hip").read().split("\n")
# function start lines in ie_resolve.hip
starts = [(i + 1, re.sub(r"\(.*", "", l).split()[-1]) for i, l in enumerate(src)
          if re.match(r"^(__device__|__global__|template|static|__launch)", l) and "(" in l]
def region(line):
    name = "?"
    for ln, nm in starts:
        if ln <= line:
            name = nm
    return name
for f in re.split(r"\n(?=_ZN2ie4r2569k_resolveI\w+:)", s):
    m = re.match(r"_ZN2ie4r2569k_resolveI(\w+)EEvNS\w+:", f)
    if not m or m.group(1) != want:
        continue
    cnt = collections.defaultdict(collections.Counter)
    cur = ("?", 0)
    for line in f.split("\n"):
        mm = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", line)
        if mm:
            fn = files.get(mm.group(1), "?").split("/")[-1]
            ln = int(mm.group(2))
            cur = (fn, ln)
            continue
        t = line.strip()
        if not t or t.startswith((".", ";")) or t.endswith(":"):
            continue
        op = t.split()[0]
        cls = "valu" if op.startswith("v_") else "salu" if op.startswith("s_") else "lds" if op.startswith("ds_") \
            else "vmem" if op.startswith(("global_", "buffer_", "flat_", "scratch_")) else "other"
        key = region(cur[1]) if cur[0] == "ie_resolve.hip" else cur[0]
        cnt[key][cls] += 1
    tot = collections.Counter()
    for k, c in sorted(cnt.items(), key=lambda kv: -sum(kv[1].values())):
        tot.update(c)
        print("%-28s %s" % (k, dict(c)))
    print("total", dict(tot))
