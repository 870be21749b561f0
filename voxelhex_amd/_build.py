"""Builds libvhx.so in-tree (voxelhex_amd/_lib/) for gfx950: host C++ with g++, HIP kernels with hipcc.

Float semantics matter for parity with the reference raytracer: every unit is compiled with -ffp-contract=off and
without fast-math (IEEE division / sqrt, f32 denormals kept on the GPU).
"""
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "_lib")
BUILD = os.path.join(ROOT, "build", "vhx")
LIB = os.path.join(LIBDIR, "libvhx.so")
# diagnostic variant builds (never loaded by the package unless VHX_LIB names them): the negative control of the tree-write
# ordering (tests/test_gpu_tuning.py), with libvhx's waits compiled out
UNORDERED_LIB = os.path.join(LIBDIR, "libvhx_unordered.so")
# ... and the chain-stamp build of scripts/chain_profile.py (VHX_CHAIN: vhx_chain_profile)
CHAIN_LIB = os.path.join(LIBDIR, "libvhx_chain.so")
ARCH = os.environ.get("VHX_OFFLOAD_ARCH", "gfx950")

HOST_SRCS = ["boxtree.cpp", "flatten.cpp", "vox.cpp", "stream.cpp"]
# device code generation: LLVM's iterative ILP scheduler for AMDGPU (instruction order and register pressure only; the
# arithmetic and its rounding are unchanged). Bench frame at eight frames in flight 0.592-0.602 ms against 0.613-0.616
# with the default scheduler; trace kernels 70 / 97 VGPRs against 75 / 102 (profiles/r02/sched_variants_f8.log)
DEV_FLAGS = ["-mllvm", "-amdgpu-sched-strategy=iterative-ilp"]
DEV_SRCS = ["vhx_device.hip", "vhx_mgpu.hip"]
HEADERS = ["boxtree.hpp", "trace.hpp", "ctx.hpp"]


def _hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build(verbose=False, force=False, lib=None, build_dir=None, defines=(), flags=(), dev_flags=None, host_flags=()):
    """lib / build_dir / defines / flags / dev_flags: a variant build (probes), e.g. defines=("VHX_QUEUE_WPE=5",),
    flags=("-O2",) added to the device sources, dev_flags=() for LLVM's default scheduler; host_flags are added to the
    host C++ sources (scripts/asan_cpu.sh: -fsanitize=address,undefined, resolved at run time from the preloaded
    sanitizer runtimes)."""
    dev = DEV_FLAGS if dev_flags is None else list(dev_flags)
    lib = lib or LIB
    bdir = build_dir or BUILD
    os.makedirs(os.path.dirname(lib), exist_ok=True)
    os.makedirs(bdir, exist_ok=True)
    dflags = [f"-D{d}" for d in defines]
    inc = os.path.join(ROOT, "include")
    common_deps = [os.path.join(inc, h) for h in ("vhx.h", "vhx_boxtree.h")] + [os.path.join(CSRC, h) for h in HEADERS]
    objs = []
    for src in HOST_SRCS:
        s = os.path.join(CSRC, src)
        o = os.path.join(bdir, src + ".o")
        if force or _stale(o, [s] + common_deps):
            _run(["g++", "-O3", "-std=c++17", "-fPIC", "-pthread", "-ffp-contract=off", "-fno-fast-math",
                  "-Wall", "-Wextra", "-I", inc] + list(host_flags) + ["-c", s, "-o", o], verbose)
        objs.append(o)
    for src in DEV_SRCS:
        s = os.path.join(CSRC, src)
        o = os.path.join(bdir, src + ".o")
        if force or _stale(o, [s] + common_deps):
            _run([_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
                  "-fno-fast-math", "-Wall", "-I", inc] + dev + dflags + list(flags) + ["-c", s, "-o", o], verbose)
        objs.append(o)
    if force or _stale(lib, objs):
        # -ldl: RCCL is dlopen()ed by vhx_mgpu.hip (no link-time RCCL dependency)
        _run([_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-pthread", "-o", lib] + objs + ["-ldl"], verbose)
    return lib


def build_variants(verbose=False, force=False):
    """The diagnostic variant libraries the GPU tests load in child processes (built here, in-tree, so they travel)."""
    build(verbose=verbose, force=force, lib=UNORDERED_LIB, build_dir=os.path.join(ROOT, "build", "vhx_unordered"),
          defines=("VHX_UNORDERED_WRITES=1",))
    build(verbose=verbose, force=force, lib=CHAIN_LIB, build_dir=os.path.join(ROOT, "build", "vhx_chain"),
          defines=("VHX_CHAIN=1",))


if __name__ == "__main__":
    build(verbose=True, force="--force" in sys.argv)
