"""Per-kernel VGPR / spill / LDS figures of a HIP source for gfx950 (from the
compiler's code-object metadata).  python tools/kstats.py FILE.hip [-DX ...] [filter]"""
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = sys.argv[1]
defs = [a for a in sys.argv[2:] if a.startswith("-D")]
filt = [a for a in sys.argv[2:] if not a.startswith("-D")]
with tempfile.TemporaryDirectory() as d:
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                    "--cuda-device-only", "-S", "-I", os.path.join(REPO, "include"),
                    "-I", os.path.join(REPO, "marl-maze_amd", "csrc"), *defs, "-o", os.path.join(d, "k.s"), src],
                   check=True)
    s = open(os.path.join(d, "k.s")).read()
meta = s[s.find("amdhsa.kernels"):]
for blk in re.split(r"\n  - ", meta)[1:]:
    def f(k):
        m = re.search(r"\." + k + r":\s+(\S+)", blk)
        return m.group(1) if m else "?"
    name = subprocess.run(["c++filt"], input=f("name"), capture_output=True, text=True).stdout.strip()
    if filt and not any(x in name for x in filt):
        continue
    print(f"vgpr {f('vgpr_count'):>4s} agpr {f('agpr_count'):>4s} spill {f('vgpr_spill_count'):>4s} "
          f"lds {f('group_segment_fixed_size'):>6s}  {name[:110]}")
