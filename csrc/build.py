"""Build the gfx950 extension in-tree with hipcc (no hipify, no setuptools
CUDA machinery): every ``csrc/kernels/*.hip`` is compiled for
``--offload-arch=gfx950`` in parallel, ``csrc/bind.cpp`` (the only TU that
includes torch headers) is compiled once, and everything is linked into
``pytorch_multiprocessing_distributed_amd/_C<EXT_SUFFIX>``.  Objects are
rebuilt only when a source or header is newer.

    python csrc/build.py [--force] [--jobs N] [--debug]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
PKG = os.path.join(ROOT, "pytorch_multiprocessing_distributed_amd")
BUILD = os.path.join(ROOT, "build", "csrc")
ARCH = os.environ.get("PMD_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _torch_paths():
    import torch
    from torch.utils import cpp_extension
    inc = cpp_extension.include_paths(device_type="cuda")
    lib = os.path.join(os.path.dirname(torch.__file__), "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def target_path():
    return os.path.join(PKG, "_C" + sysconfig.get_config_var("EXT_SUFFIX"))


def _newer(src_files, out):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(s) > t for s in src_files)


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}):\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return r


ASAN_DIR = os.path.join(ROOT, "build", "asan")
ASAN_FLAGS = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fno-omit-frame-pointer"]


def asan_runtime():
    """Path of the clang ASan runtime to LD_PRELOAD into Python (host code only)."""
    r = subprocess.run([HIPCC, "-print-file-name=libclang_rt.asan-x86_64.so"], capture_output=True, text=True)
    p = r.stdout.strip()
    return p if r.returncode == 0 and os.path.isabs(p) and os.path.exists(p) else None


def build(force=False, jobs=None, debug=False, verbose=True, asan=False):
    """asan=True: the host C++ (binding layer + native runtime: reducer, RCCL/xGMI
    communicators, weight-image sets) instrumented with AddressSanitizer
    (-Xarch_host only: GPU code is never sanitised), device kernels reused, the
    library written to build/asan/ -- load it with PMD_EXT_DIR=build/asan and
    the ASan runtime preloaded (tests/test_asan_cpu.py)."""
    os.makedirs(BUILD, exist_ok=True)
    inc, lib, abi = _torch_paths()
    headers = glob.glob(os.path.join(CSRC, "kernels", "*.h"))
    opt = ["-O1", "-g"] if (debug or asan) else ["-O3"]
    common = [HIPCC, f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", *opt,
              "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
              *os.environ.get("PMD_EXTRA_CFLAGS", "").split()]  # A/B variant macros
    jobs_ = []
    objs = []
    kcommon = [HIPCC, f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-O3",
               "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
               *os.environ.get("PMD_EXTRA_CFLAGS", "").split()]
    for src in sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip"))):
        obj = os.path.join(BUILD, os.path.basename(src) + ".o")   # shared by the ASan build
        objs.append(obj)
        if force or _newer([src, *headers], obj):
            jobs_.append((kcommon if asan else common) + ["-c", src, "-o", obj,
                                                          f"-I{os.path.join(CSRC, 'kernels')}"])
    hbuild = os.path.join(ROOT, "build", "csrc_asan") if asan else BUILD
    os.makedirs(hbuild, exist_ok=True)
    # host TUs that include torch headers: the binding layer + native runtime
    # (reducer, comm bootstrap); they are host-only C++ compiled by hipcc
    torch_tus = [os.path.join(CSRC, "bind.cpp")] + sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    rt_headers = glob.glob(os.path.join(CSRC, "runtime", "*.h"))
    for src in torch_tus:
        obj = os.path.join(hbuild, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or _newer([src, *headers, *rt_headers], obj):
            jobs_.append(common + (ASAN_FLAGS if asan else []) + [
                "-x", "hip", "-c", src, "-o", obj, f"-I{CSRC}",
                *[f"-I{p}" for p in inc], f"-I{sysconfig.get_paths()['include']}",
                "-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H",
                f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-Wno-unused-result", "-Wno-deprecated-declarations"])
    if jobs_:
        n = jobs or min(len(jobs_), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 16)
        if verbose:
            print(f"[pmd build] compiling {len(jobs_)} TU(s) for {ARCH} with {n} job(s)", flush=True)
        with cf.ThreadPoolExecutor(n) as ex:
            for f in [ex.submit(_run, j) for j in jobs_]:
                f.result()
    out = target_path()
    if asan:
        os.makedirs(ASAN_DIR, exist_ok=True)
        out = os.path.join(ASAN_DIR, os.path.basename(out))
    if force or jobs_ or _newer(objs, out):
        link = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out, *objs,
                *(["-Xarch_host", "-fsanitize=address", "-shared-libsan"] if asan else []),
                f"-L{lib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
                "-ltorch_python", "-l:librccl.so", f"-Wl,-rpath,{lib}",
                "-L/opt/rocm/lib", "-lrocprofiler-sdk-roctx", "-Wl,-rpath,/opt/rocm/lib"]
        _run(link)
        if verbose:
            print(f"[pmd build] linked {out}", flush=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=None)
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("--asan", action="store_true", help="host-side AddressSanitizer build -> build/asan/")
    a = ap.parse_args()
    build(force=a.force, jobs=a.jobs, debug=a.debug, asan=a.asan)


if __name__ == "__main__":
    sys.exit(main())
