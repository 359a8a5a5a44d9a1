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
# A/B timing builds only (tools/gpu/iter.sh): TBGPU_TIMING_KNOBS=1 compiles in the TBGPU_ABLATE /
# TBGPU_FLOW_GRID / TBGPU_NO_FLOW / TBGPU_ACCOUNT_SLOTS environment knobs (csrc/pass.h TB_ABL).
if os.environ.get("TBGPU_TIMING_KNOBS") == "1":
    FLAGS.append("-DTBGPU_TIMING_KNOBS")


def _sources():
    inc = os.path.join(ROOT, "include")
    return [os.path.join(CSRC, f) for f in sorted(os.listdir(CSRC)) if f.endswith((".hip", ".h"))] + [
        os.path.join(inc, f) for f in sorted(os.listdir(inc)) if f.endswith(".h")]


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


HOST = os.path.join(PKG_DIR, "host")
RUNNER = os.path.join(HOST, "tb_table_runner")
CXX = os.environ.get("CXX", shutil.which("g++") or "g++")


def build_host(force=False, verbose=True):
    """The C++ host mirror (host/state_machine.*) and its golden-table runner, linked against the
    in-tree engine (rpath $ORIGIN/..)."""
    srcs = [os.path.join(HOST, f) for f in ("state_machine.cpp", "table_runner.cpp")]
    deps = srcs + [os.path.join(HOST, "state_machine.hpp"), os.path.join(ROOT, "include", "tbgpu.h"), LIB]
    if not force and not _stale(RUNNER, deps):
        return RUNNER
    cmd = [CXX, "-O2", "-std=c++17", "-Wall", "-Wextra", "-o", RUNNER + ".tmp"] + srcs + [
        "-L" + PKG_DIR, "-ltbgpu", "-Wl,-rpath,$ORIGIN/.."]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(RUNNER + ".tmp", RUNNER)
    return RUNNER


REPLICA_BENCH = os.path.join(HOST, "tb_replica_bench")


def build_replica_bench(force=False, verbose=True):
    """tb_replica_bench: the replica's call path (prepare -> prefetch -> commit -> compact) through the
    C++ mirror, for bench.py's replica_path leg."""
    srcs = [os.path.join(HOST, f) for f in ("state_machine.cpp", "replica_bench.cpp")]
    deps = srcs + [os.path.join(HOST, "state_machine.hpp"), os.path.join(ROOT, "include", "tbgpu.h"),
                   os.path.join(ROOT, "include", "tbgpu_bench.h"), LIB]
    if not force and not _stale(REPLICA_BENCH, deps):
        return REPLICA_BENCH
    cmd = [CXX, "-O2", "-std=c++17", "-Wall", "-Wextra", "-o", REPLICA_BENCH + ".tmp"] + srcs + [
        "-L" + PKG_DIR, "-ltbgpu", "-Wl,-rpath,$ORIGIN/.."]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(REPLICA_BENCH + ".tmp", REPLICA_BENCH)
    return REPLICA_BENCH


def build(force=False, verbose=True):
    lib = build_engine(force=force, verbose=verbose)
    build_host(force=force, verbose=verbose)
    build_replica_bench(force=force, verbose=verbose)
    return lib


if __name__ == "__main__":
    build(force="--force" in sys.argv)
