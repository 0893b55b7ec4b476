"""Build libsrk.so in-tree with hipcc for gfx950 (no JIT cache: the .so travels to the GPU box).

    python -m speechrecognitionproject_amd.build [--force] [-j N]
"""
import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
BUILD = os.path.join(PKG, "_build")
LIB = os.path.join(PKG, "libsrk.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
         "-mllvm", "-disable-promote-alloca-to-lds",   # private arrays stay in VGPRs, never silently in LDS
         "-Wall", "-Wno-unused-function", "-Wno-unused-variable", "-I", os.path.join(REPO, "include")]


def _sources():
    # *.hip: device + host code; *.cpp: host-only code (input pipeline), same compiler and flags
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))


def _headers():
    return sorted(glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(REPO, "include", "*.h")))


def _compile(src, force):
    obj = os.path.join(BUILD, os.path.basename(src) + ".o")
    deps = [src] + _headers()
    if not force and os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(d) for d in deps):
        return obj, False
    cmd = [HIPCC, *FLAGS, "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("hipcc failed for %s:\n%s\n%s" % (src, " ".join(cmd), r.stderr))
    return obj, True


def build(force=False, jobs=None, verbose=True):
    """Compile every csrc/*.hip (+ host-only *.cpp) for gfx950 and link libsrk.so; returns its path."""
    os.makedirs(BUILD, exist_ok=True)
    srcs = _sources()
    jobs = jobs or min(len(srcs), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 16)
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        results = list(ex.map(lambda s: _compile(s, force), srcs))
    objs = [o for o, _ in results]
    rebuilt = any(r for _, r in results)
    if rebuilt or force or not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(o) for o in objs):
        tmp = LIB + ".tmp"
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", tmp]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("link failed:\n%s\n%s" % (" ".join(cmd), r.stderr))
        os.replace(tmp, LIB)
        if verbose:
            print("built", LIB, file=sys.stderr)
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=None)
    a = ap.parse_args()
    build(force=a.force, jobs=a.j)
