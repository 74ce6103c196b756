"""Native build: hipcc for gfx950, in-tree outputs (they travel to the GPU box).

    libsgufp_hip.so   kernels + C ABI (include/sgufp_hip.h), linked with RCCL (frontier shards)
    lib_verify/libsgufp_hip.so
                      the same with SGUFP_SUB_VERIFY: every warm-started Bellman-Ford of the
                      subproblem is re-run cold and compared (debug build for tests)
    lib_prof/libsgufp_hip.so
                      the same with k_relax's per-wave clock stamps (SGUFP_PHASES) for the
                      diagnostics tools; the production kernel carries none
    libsgufp_host.so  C++ mirror of the reference's host API (Network / NodeExplorer /
                      GuroSolver / DDSolver, include/sgufp/inavap.hpp) on top of the C ABI
    host_api_test     C++ driver of that API (tests/host/host_api_test.cpp)
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "lib")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

COMMON = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-Wall", "-Wno-unused-function",
          f"-I{os.path.join(ROOT, 'include')}", f"-I{CSRC}"]

HIP_SOURCES = ["dd_kernels.hip", "sub_kernels.hip", "bnb_kernels.hip", "rdd_kernels.hip", "exact_kernels.hip", "capi.cpp",
               "bnb.cpp", "network.cpp", "shard.cpp"]
LINK = ["-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]   # frontier shards (shard.cpp)
HOST_SOURCES = ["host/inavap.cpp"]


def _run(cmd, cwd=None):
    r = subprocess.run(cmd, cwd=cwd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError(f"build failed: {' '.join(cmd)}")
    return r


def _stale(target, sources):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in sources)


def build_native(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(LIBDIR, exist_ok=True)
    objdir = os.path.join(LIBDIR, "obj")
    os.makedirs(objdir, exist_ok=True)
    headers = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hpp", ".h"))]
    headers.append(os.path.join(ROOT, "include", "sgufp_hip.h"))
    objs = []
    for src in HIP_SOURCES:
        path = os.path.join(CSRC, src)
        obj = os.path.join(objdir, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or _stale(obj, [path] + headers):
            lang = ["-x", "hip"] if src.endswith(".hip") else []
            cmd = [HIPCC, f"--offload-arch={ARCH}", *COMMON, *lang, "-c", path, "-o", obj]
            if verbose:
                print(" ".join(cmd))
            _run(cmd)
    lib = os.path.join(LIBDIR, "libsgufp_hip.so")
    if force or _stale(lib, objs):
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib, *objs, *LINK])
    # debug variant: subproblem kernels with the warm Bellman-Ford cross-check
    vdir = os.path.join(HERE, "lib_verify")
    os.makedirs(vdir, exist_ok=True)
    vsrc = os.path.join(CSRC, "sub_kernels.hip")
    vobj = os.path.join(objdir, "sub_kernels_verify.o")
    if force or _stale(vobj, [vsrc] + headers):
        _run([HIPCC, f"--offload-arch={ARCH}", *COMMON, "-DSGUFP_SUB_VERIFY", "-x", "hip", "-c", vsrc, "-o", vobj])
    vlib = os.path.join(vdir, "libsgufp_hip.so")
    vobjs = [vobj if os.path.basename(o) == "sub_kernels.hip.o" else o for o in objs]
    if force or _stale(vlib, vobjs):
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", vlib, *vobjs, *LINK])
    # profiling variant: k_relax with its per-wave / per-phase clock stamps (tools/*_diag.py)
    pdir = os.path.join(HERE, "lib_prof")
    os.makedirs(pdir, exist_ok=True)
    psrc = os.path.join(CSRC, "dd_kernels.hip")
    pobj = os.path.join(objdir, "dd_kernels_prof.o")
    if force or _stale(pobj, [psrc] + headers):
        _run([HIPCC, f"--offload-arch={ARCH}", *COMMON, "-DSGUFP_PHASES", "-x", "hip", "-c", psrc, "-o", pobj])
    plib = os.path.join(pdir, "libsgufp_hip.so")
    pobjs = [pobj if os.path.basename(o) == "dd_kernels.hip.o" else o for o in objs]
    if force or _stale(plib, pobjs):
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", plib, *pobjs, *LINK])
    host_srcs = [os.path.join(CSRC, s) for s in HOST_SOURCES if os.path.exists(os.path.join(CSRC, s))]
    if host_srcs:
        hlib = os.path.join(LIBDIR, "libsgufp_host.so")
        hheaders = [os.path.join(ROOT, "include", "sgufp", f) for f in os.listdir(os.path.join(ROOT, "include", "sgufp"))] \
            if os.path.isdir(os.path.join(ROOT, "include", "sgufp")) else []
        if force or _stale(hlib, host_srcs + hheaders + [lib]):
            cxx = shutil.which("g++") or "g++"
            _run([cxx, "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", f"-I{os.path.join(ROOT, 'include')}",
                  *host_srcs, "-o", hlib, f"-L{LIBDIR}", "-lsgufp_hip", "-Wl,-rpath,$ORIGIN"])
        # C++ driver of the host API used by tests/test_host_api.py
        tsrc = os.path.join(ROOT, "tests", "host", "host_api_test.cpp")
        texe = os.path.join(LIBDIR, "host_api_test")
        if os.path.exists(tsrc) and (force or _stale(texe, [tsrc, hlib] + hheaders)):
            cxx = shutil.which("g++") or "g++"
            _run([cxx, "-O2", "-std=c++17", "-Wall", f"-I{os.path.join(ROOT, 'include')}", tsrc, "-o", texe,
                  f"-L{LIBDIR}", "-lsgufp_host", "-lsgufp_hip", "-Wl,-rpath,$ORIGIN"])
    return lib


if __name__ == "__main__":
    print(build_native(force="--force" in sys.argv, verbose=True))
