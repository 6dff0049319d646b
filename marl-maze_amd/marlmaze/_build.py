"""Build libmarlmaze.so in-tree with hipcc for gfx950 (no cmake, no JIT cache)."""
import glob
import os
import subprocess

from ._paths import PKG_ROOT, REPO_ROOT

CSRC = os.path.join(PKG_ROOT, "csrc")
LIB = os.path.join(PKG_ROOT, "libmarlmaze.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-std=c++17",
         "-ffp-contract=off",  # the reference's fp32 op order (GAE) must not fuse into FMA
         "-Wall", "-Wno-unused-result"]


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def needs_build():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = sources() + glob.glob(os.path.join(CSRC, "*.h")) + [os.path.join(REPO_ROOT, "include", "marlmaze.h")]
    return any(os.path.getmtime(p) > t for p in deps)


def build(force=False, verbose=False):
    if not force and not needs_build():
        return LIB
    cmd = [HIPCC] + FLAGS + ["-I", os.path.join(REPO_ROOT, "include"), "-I", CSRC, "-o", LIB + ".tmp"] + sources()
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(LIB + ".tmp", LIB)
    return LIB
