"""Builds the native extension `mpi_tensorflow_amd/_C*.so` in-tree with hipcc.

Every HIP source is compiled for gfx950 only (`--offload-arch=gfx950`); host
C++ (RCCL loader, IDX reader, executor, bindings) goes through the same
hipcc driver.  The link pulls libamdhip64 by soname, which resolves to the
runtime the PyTorch-ROCm wheel has already loaded when `import torch` runs
first (the package always imports torch before `_C`).

    python -m mpi_tensorflow_amd.build_ext [--force] [-j N] [-v]
"""

from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig
import time

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
BUILD = os.path.join(ROOT, "build", "native")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0] or "gfx950"


def ext_path() -> str:
    return os.path.join(PKG, "_C" + sysconfig.get_config_var("EXT_SUFFIX"))


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc"):
        if c and os.path.exists(c):
            return c
    return "hipcc"


def _sources():
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.cpp")) + glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    return srcs


def _headers():
    return sorted(glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True))


def _flags():
    import pybind11

    inc = [CSRC, pybind11.get_include(), sysconfig.get_paths()["include"]]
    f = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wno-unused-result",
         "-fvisibility=hidden", "-D__HIP_PLATFORM_AMD__"]
    for i in inc:
        f += ["-I", i]
    return f


def _obj(src: str) -> str:
    rel = os.path.relpath(src, CSRC).replace(os.sep, "_")
    return os.path.join(BUILD, rel + ".o")


def _stale(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, jobs: int = 0, verbose: bool = False) -> str:
    """Compiles stale objects in parallel and links the extension; returns its path."""
    os.makedirs(BUILD, exist_ok=True)
    hipcc = _hipcc()
    flags = _flags()
    hdrs = _headers()
    srcs = _sources()
    todo = [s for s in srcs if force or _stale(_obj(s), [s] + hdrs + [__file__])]
    jobs = jobs or min(8, os.cpu_count() or 4)

    def compile_one(src):
        lang = ["-x", "hip"] if src.endswith(".hip") else []
        cmd = [hipcc] + lang + flags + ["-c", src, "-o", _obj(src)]
        t0 = time.time()
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        if verbose:
            print(f"  compiled {os.path.relpath(src, ROOT)} in {time.time() - t0:.1f}s", flush=True)

    if todo:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            list(ex.map(compile_one, todo))
    out = ext_path()
    objs = [_obj(s) for s in srcs]
    if force or todo or _stale(out, objs):
        cmd = [hipcc, "-shared", f"--offload-arch={ARCH}", "-o", out] + objs + ["-lz", "-ldl"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        if verbose:
            print(f"  linked {os.path.relpath(out, ROOT)}", flush=True)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=0)
    ap.add_argument("-v", action="store_true")
    a = ap.parse_args(argv)
    t0 = time.time()
    p = build(a.force, a.j, a.v)
    print(f"built {p} in {time.time() - t0:.1f}s")


if __name__ == "__main__":
    sys.exit(main())
