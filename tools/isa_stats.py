"""Per-kernel ISA statistics of a HIP source compiled for gfx950 (instruction mix, VGPRs, LDS)."""
import collections
import os
import re
import subprocess
import sys
import tempfile

src = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else ""
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
with tempfile.TemporaryDirectory() as d:
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-mcode-object-version=5"] + os.environ.get("ISA_FLAGS", "").split() + [
                    "--cuda-device-only", "-S", "-o", os.path.join(d, "k.s"), src], check=True)
    s = open(os.path.join(d, "k.s")).read()
meta = dict(re.findall(r"\.name:\s+(\S+)\n(?:.*\n){0,40}?\s+\.vgpr_count:\s+(\d+)", s))
for m in re.finditer(r"^(\S+):\s*;\s*@\1\n(.*?)^\.Lfunc_end", s, re.S | re.M):
    name, body = m.group(1), m.group(2)
    if pat not in name:
        continue
    ins = [l.split()[0] for l in body.split("\n") if l.startswith("\t") and l.strip() and not l.strip().startswith((".", ";"))]
    c = collections.Counter(ins)
    print(f"{name[:90]}: {len(ins)} instr, vgpr={meta.get(name, '?')}")
    print("   ", ", ".join(f"{k}:{v}" for k, v in c.most_common(25)))
