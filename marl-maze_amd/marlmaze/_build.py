"""Build libmarlmaze.so in-tree with hipcc for gfx950 (no cmake, no JIT cache).

Next to the library, build() writes ``libmarlmaze.so.srcsha``: the sha256 of the
compile flags and of every source and header the library is built from.  The
loader (marlmaze._lib) recomputes it and refuses a library whose sources have
changed since it was built, so a stale prebuilt binary that travels to the GPU
box with the tree cannot be tested silently.
"""
import glob
import hashlib
import os
import subprocess

from ._paths import PKG_ROOT, REPO_ROOT

CSRC = os.path.join(PKG_ROOT, "csrc")
LIB = os.path.join(PKG_ROOT, "libmarlmaze.so")
HASH_FILE = LIB + ".srcsha"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-std=c++17",
         "-ffp-contract=off",  # the reference's fp32 op order (GAE) must not fuse into FMA
         "-Wall", "-Wno-unused-result"]


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def deps():
    return sources() + sorted(glob.glob(os.path.join(CSRC, "*.h"))) + [os.path.join(REPO_ROOT, "include",
                                                                                   "marlmaze.h")]


def source_hash():
    """sha256 over the flags and the (name, bytes) of every dependency."""
    h = hashlib.sha256(" ".join(FLAGS).encode())
    for p in deps():
        h.update(b"\0" + os.path.basename(p).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def stored_hash():
    try:
        with open(HASH_FILE) as f:
            return f.read().strip()
    except OSError:
        return None


def needs_build():
    return not os.path.exists(LIB) or stored_hash() != source_hash()


def build(force=False, verbose=False):
    if not force and not needs_build():
        return LIB
    digest = source_hash()  # of the sources as compiled (an edit during the build makes the result stale)
    cmd = [HIPCC] + FLAGS + ["-I", os.path.join(REPO_ROOT, "include"), "-I", CSRC, "-o", LIB + ".tmp"] + sources()
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(LIB + ".tmp", LIB)
    with open(HASH_FILE + ".tmp", "w") as f:
        f.write(digest + "\n")
    os.replace(HASH_FILE + ".tmp", HASH_FILE)
    return LIB
