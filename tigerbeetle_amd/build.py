"""Build the in-tree HIP engine (libtbgpu.so) for gfx950 and the C++ host-side tools.

    python -m tigerbeetle_amd.build            # engine + host tools
"""
import os
import shutil
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG_DIR)
CSRC = os.path.join(PKG_DIR, "csrc")
LIB = os.path.join(PKG_DIR, "libtbgpu.so")

HIPCC = os.environ.get("HIPCC", shutil.which("hipcc") or "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
FLAGS = ["--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-Wall", "-Werror=return-type"]


def _sources():
    return [os.path.join(CSRC, f) for f in sorted(os.listdir(CSRC)) if f.endswith((".hip", ".h"))] + [
        os.path.join(ROOT, "include", "tbgpu.h"), os.path.join(ROOT, "include", "tbgpu_bench.h")]


def _stale(target, sources):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in sources)


def build_engine(force=False, verbose=True):
    if not force and not _stale(LIB, _sources()):
        return LIB
    cmd = [HIPCC] + FLAGS + ["-shared", "-o", LIB + ".tmp", os.path.join(CSRC, "engine.hip")]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(LIB + ".tmp", LIB)
    return LIB


def build(force=False, verbose=True):
    return build_engine(force=force, verbose=verbose)


if __name__ == "__main__":
    build(force="--force" in sys.argv)
