"""Build libmarlmaze.so variants for in-process A/B timing (tools/ab_libs.py):
  python tools/ab_build.py base [REV]   -> tools/_var/base.so from the csrc/ of git REV (default HEAD)
  python tools/ab_build.py NAME [-DX..]  -> tools/_var/NAME.so from the working tree (extra defines)"""
import os
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"
FLAGS = ["--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-std=c++17", "-ffp-contract=off", "-w"]


def build(name, csrc, include, defs=()):
    out = os.path.join(REPO, "tools", "_var", name + ".so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    srcs = sorted(os.path.join(csrc, f) for f in os.listdir(csrc) if f.endswith(".hip"))
    subprocess.run([HIPCC, *FLAGS, *defs, "-I", include, "-I", csrc, "-o", out, *srcs], check=True)
    print(out)


if __name__ == "__main__":
    name = sys.argv[1]
    if name == "base":
        rev = sys.argv[2] if len(sys.argv) > 2 else "HEAD"
        with tempfile.TemporaryDirectory() as d:
            for sub in ("marl-maze_amd/csrc", "include"):
                os.makedirs(os.path.join(d, sub), exist_ok=True)
                files = subprocess.run(["git", "-C", REPO, "ls-tree", "--name-only", rev, sub + "/"], check=True,
                                       capture_output=True, text=True).stdout.split()
                for f in files:
                    data = subprocess.run(["git", "-C", REPO, "show", f"{rev}:{f}"], check=True,
                                          capture_output=True).stdout
                    open(os.path.join(d, f), "wb").write(data)
            build("base", os.path.join(d, "marl-maze_amd/csrc"), os.path.join(d, "include"))
    else:
        build(name, os.path.join(REPO, "marl-maze_amd", "csrc"), os.path.join(REPO, "include"), sys.argv[2:])
