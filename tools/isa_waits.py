"""Map the vmcnt waits / scratch accesses of a kernel's gfx950 ISA to source lines.

Usage: python tools/isa_waits.py FILE.hip KERNEL_SUBSTRING
(offline, no GPU: compiles with line tables and prints, per source line, the count
of `s_waitcnt vmcnt(k)` for small k (<= 2) and of scratch instructions.)
"""
import collections
import os
import re
import subprocess
import sys
import tempfile

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src, kern = sys.argv[1], sys.argv[2]
out = os.path.join(tempfile.mkdtemp(), "k.s")
subprocess.run(["/opt/rocm/bin/hipcc", "-std=c++17", "-O3", "-gline-tables-only", "--offload-arch=gfx950",
                "--cuda-device-only", "-S", "-I", os.path.join(R, "pino-locoman_amd/csrc"), "-I",
                os.path.join(R, "include"), src, "-o", out], check=True, capture_output=True)
s = open(out).read()
names = re.findall(r"^(_Z\w*" + kern + r"\w*):", s, re.M)
k = s.index(names[0] + ":")
body = s[k:s.index(".Lfunc_end", k)].split("\n")
lines = open(src).read().split("\n")
files = dict(re.findall(r'^\s*\.file\s+(\d+)\s+"[^"]*"\s+"([^"]+)"', s, re.M))
main_file = next((int(k) for k, v in files.items() if v.endswith(os.path.basename(src))), 0)
cur = 0
waits, scr = collections.Counter(), collections.Counter()
for l in body:
    m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)\s+", l)
    if m:
        cur = int(m.group(2)) if int(m.group(1)) == main_file else -1
        continue
    t = l.strip()
    m = re.match(r"s_waitcnt.*vmcnt\((\d+)\)", t)
    if m and int(m.group(1)) <= 2:
        waits[cur] += 1
    if t.startswith("scratch"):
        scr[cur] += 1
print(names[0])
for ln, c in sorted(waits.items()):
    print(f"vmcnt<=2 x{c:3d}  {ln:5d}  {lines[ln - 1].strip()[:100] if ln > 0 else '(other file)'}")
for ln, c in sorted(scr.items()):
    print(f"scratch  x{c:3d}  {ln:5d}  {lines[ln - 1].strip()[:100] if ln > 0 else '(other file)'}")
