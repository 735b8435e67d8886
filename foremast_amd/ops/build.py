"""Build the gfx950 HIP kernels into one in-tree shared library.

``python -m foremast_amd.ops.build`` compiles every ``csrc/*.hip`` with
``hipcc --offload-arch=gfx950`` (incrementally, in parallel) and links
``_lib/libforemast_hip.so``.  No torch headers are involved: the kernels
expose a C ABI (``extern "C" fm_*``) that :mod:`foremast_amd.ops._native`
binds with ctypes and launches on the current PyTorch HIP stream.  The
library is built in-tree so it travels with the repository snapshot to the
GPU box.
"""

from __future__ import annotations

import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from typing import List

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "_lib")
BUILDDIR = os.path.join(LIBDIR, "obj")
LIBNAME = "libforemast_hip.so"
ARCH = os.environ.get("FOREMAST_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm toolchain required to build the kernels)")


def _flags() -> List[str]:
    return ["-O3", f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-ffp-contract=fast",
            "-munsafe-fp-atomics", "-Wno-unused-result", "-Werror=return-type"]


def sources() -> List[str]:
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))


def headers() -> List[str]:
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h"))


def lib_path() -> str:
    # FOREMAST_HIP_LIB: load another build of the library (same-box A/B of a kernel change)
    return os.environ.get("FOREMAST_HIP_LIB") or os.path.join(LIBDIR, LIBNAME)


def _needs(obj: str, deps: List[str]) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in deps)


def build(verbose: bool = False, jobs: int = 8) -> str:
    os.makedirs(BUILDDIR, exist_ok=True)
    cc = hipcc()
    hdrs = headers()
    objs = []
    todo = []
    for src in sources():
        obj = os.path.join(BUILDDIR, os.path.basename(src)[:-4] + ".o")
        objs.append(obj)
        if _needs(obj, [src] + hdrs):
            todo.append((src, obj))

    def compile_one(pair):
        src, obj = pair
        cmd = [cc, *_flags(), "-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
        return obj

    if todo:
        with ThreadPoolExecutor(max_workers=max(1, min(jobs, len(todo)))) as ex:
            list(ex.map(compile_one, todo))
    lib = lib_path()
    if todo or not os.path.exists(lib) or _needs(lib, objs):
        tmp = lib + ".tmp"
        cmd = [cc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *objs]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")
        os.replace(tmp, lib)
    return lib


if __name__ == "__main__":
    path = build(verbose="-v" in sys.argv)
    print(path)
