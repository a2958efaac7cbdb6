"""Build the gfx950 extension in-tree with hipcc (no hipify, no setuptools
CUDA machinery): every ``csrc/kernels/*.hip`` is compiled for
``--offload-arch=gfx950`` in parallel, ``csrc/bind.cpp`` (the only TU that
includes torch headers) is compiled once, and everything is linked into
``pytorch_multiprocessing_distributed_amd/_C<EXT_SUFFIX>``.  Every object carries a
sha256 stamp of its sources' CONTENTS and its compile command, and is rebuilt
exactly when that changes (never on file mtimes); the library is relinked when any
object changed, and ``_C.stamp.json`` records the source hash, the arch and the
flags, which the loader (ops/native.py) checks against the tree at import.

    python csrc/build.py [--force] [--jobs N] [--debug]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import hashlib
import json
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


def _digest(paths, flags):
    """sha256 over the CONTENTS of ``paths`` (sorted, with their names) and the
    compile command ``flags``: build provenance that does not depend on file mtimes
    (a copied tree, a checkout or a touched file cannot make a stale object look fresh)."""
    h = hashlib.sha256()
    for pth in sorted(paths):
        h.update(os.path.relpath(pth, ROOT).encode() + b"\0")
        with open(pth, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    h.update("\0".join(flags).encode())
    return h.hexdigest()


def _stale(digest, out):
    """True unless ``out`` exists and its ``.sha256`` stamp records ``digest``."""
    stamp = out + ".sha256"
    if not (os.path.exists(out) and os.path.exists(stamp)):
        return True
    with open(stamp) as f:
        return f.read().strip() != digest


def _stamp(out, digest):
    with open(out + ".sha256", "w") as f:
        f.write(digest + "\n")


def source_files():
    """Every file the extension is built from (kernels, headers, bindings, runtime)."""
    return (glob.glob(os.path.join(CSRC, "kernels", "*.hip")) + glob.glob(os.path.join(CSRC, "kernels", "*.h"))
            + [os.path.join(CSRC, "bind.cpp")] + glob.glob(os.path.join(CSRC, "runtime", "*.cpp"))
            + glob.glob(os.path.join(CSRC, "runtime", "*.h")))


def source_digest():
    """Content hash of the extension's sources alone (no flags): what the library stamp
    records as ``sources`` and what the loader (ops/native.py) checks at import."""
    return _digest(source_files(), [])


def stamp_path():
    return os.path.join(PKG, "_C.stamp.json")


def read_stamp():
    try:
        with open(stamp_path()) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


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


def build(force=False, jobs=None, debug=False, verbose=True, asan=False, variant=None):
    """asan=True: the host C++ (binding layer + native runtime: reducer, RCCL/xGMI
    communicators, weight-image sets) instrumented with AddressSanitizer
    (-Xarch_host only: GPU code is never sanitised), device kernels reused, the
    library written to build/asan/ -- load it with PMD_EXT_DIR=build/asan and
    the ASan runtime preloaded (tests/test_asan_cpu.py)."""
    # variant="<name>": an A/B build with PMD_EXTRA_CFLAGS into build/variant_<name>/ and
    # abso/so_<name>.so (bench/ab_so.sh), leaving the production objects, library and stamp alone
    bdir = os.path.join(ROOT, "build", f"variant_{variant}") if variant else BUILD
    os.makedirs(bdir, exist_ok=True)
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
    stamps = []
    for src in sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip"))):
        obj = os.path.join(bdir, os.path.basename(src) + ".o")   # shared by the ASan build
        objs.append(obj)
        cmd = (kcommon if asan else common) + ["-c", src, "-o", obj, f"-I{os.path.join(CSRC, 'kernels')}"]
        d = _digest([src, *headers], cmd)
        if force or _stale(d, obj):
            jobs_.append(cmd)
            stamps.append((obj, d))
    hbuild = os.path.join(ROOT, "build", "csrc_asan") if asan else bdir
    os.makedirs(hbuild, exist_ok=True)
    # host TUs that include torch headers: the binding layer + native runtime
    # (reducer, comm bootstrap); they are host-only C++ compiled by hipcc
    torch_tus = [os.path.join(CSRC, "bind.cpp")] + sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    rt_headers = glob.glob(os.path.join(CSRC, "runtime", "*.h"))
    for src in torch_tus:
        obj = os.path.join(hbuild, os.path.basename(src) + ".o")
        objs.append(obj)
        cmd = common + (ASAN_FLAGS if asan else []) + [
            "-x", "hip", "-c", src, "-o", obj, f"-I{CSRC}",
            *[f"-I{p}" for p in inc], f"-I{sysconfig.get_paths()['include']}",
            "-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H",
            f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-Wno-unused-result", "-Wno-deprecated-declarations"]
        d = _digest([src, *headers, *rt_headers], cmd)
        if force or _stale(d, obj):
            jobs_.append(cmd)
            stamps.append((obj, d))
    if jobs_:
        n = jobs or min(len(jobs_), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 16)
        if verbose:
            print(f"[pmd build] compiling {len(jobs_)} TU(s) for {ARCH} with {n} job(s)", flush=True)
        with cf.ThreadPoolExecutor(n) as ex:
            for f in [ex.submit(_run, j) for j in jobs_]:
                f.result()
        for obj, d in stamps:          # only after every compile succeeded
            _stamp(obj, d)
    out = target_path()
    if variant:
        os.makedirs(os.path.join(ROOT, "abso"), exist_ok=True)
        out = os.path.join(ROOT, "abso", f"so_{variant}.so")
    if asan:
        os.makedirs(ASAN_DIR, exist_ok=True)
        out = os.path.join(ASAN_DIR, os.path.basename(out))
    obj_stamps = []
    for o in objs:
        with open(o + ".sha256") as f:
            obj_stamps.append(f.read().strip())
    lib_digest = hashlib.sha256("\n".join(obj_stamps).encode()).hexdigest()
    if force or jobs_ or _stale(lib_digest, out):
        link = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out, *objs,
                *(["-Xarch_host", "-fsanitize=address", "-shared-libsan"] if asan else []),
                f"-L{lib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
                "-ltorch_python", "-l:librccl.so", f"-Wl,-rpath,{lib}",
                "-L/opt/rocm/lib", "-lrocprofiler-sdk-roctx", "-Wl,-rpath,/opt/rocm/lib"]
        _run(link)
        _stamp(out, lib_digest)
        if verbose:
            print(f"[pmd build] linked {out}", flush=True)
    if not asan and not variant:
        st = read_stamp()
        want = {"sources": source_digest(), "library": lib_digest, "arch": ARCH,
                "opt": opt, "extra_cflags": os.environ.get("PMD_EXTRA_CFLAGS", "")}
        if st is None or any(st.get(k) != v for k, v in want.items()):
            with open(stamp_path(), "w") as f:
                json.dump(want, f, indent=1)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=None)
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("--asan", action="store_true", help="host-side AddressSanitizer build -> build/asan/")
    ap.add_argument("--variant", default=None,
                    help="A/B variant name: PMD_EXTRA_CFLAGS build -> abso/so_<name>.so (production untouched)")
    a = ap.parse_args()
    build(force=a.force, jobs=a.jobs, debug=a.debug, asan=a.asan, variant=a.variant)


if __name__ == "__main__":
    sys.exit(main())
