"""Build ``libtdq_hip.so`` (all HIP kernels, gfx950 only) in-tree with hipcc.

    python -m tensordiffeq_amd.csrc.build [--force] [-j N]

Each ``*.hip`` is compiled to an object in ``csrc/build/``, then everything is linked into
``csrc/libtdq_hip.so``.  No torch headers are involved: the kernels export a C ABI that
:mod:`tensordiffeq_amd.ops._lib` loads with ctypes.

Staleness is decided by content, not mtimes: an object is rebuilt unless the stamp next to it
(``<obj>.stamp``) holds the sha256 of its source, every header and the compile command; the
library embeds :func:`source_hash` (all ``*.hip`` + ``*.h``) through a generated
``tdq_src_hash()``, and the loader refuses a library whose hash differs from the sources beside it
(``TDQ_SKIP_HASH_CHECK=1`` overrides) - a stale ``.so`` can no longer travel to the GPU box.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import hashlib
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "libtdq_hip.so")
BUILD = os.path.join(HERE, "build")
ARCH = os.environ.get("TDQ_OFFLOAD_ARCH", "gfx950")


def hipcc():
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found")


def _flags(defines=()):
    return (["-O3", "-std=c++17", f"--offload-arch={ARCH}", "-fPIC", "-munsafe-fp-atomics", "-fno-slp-vectorize",
             "-Wno-unused-result", "-I", HERE] + [f"-D{m}" for m in defines])


def source_files():
    return sorted(glob.glob(os.path.join(HERE, "*.hip")) + glob.glob(os.path.join(HERE, "*.h")))


def source_hash():
    """sha256 (hex, 16 chars) over the names and contents of every ``*.hip`` / ``*.h`` in csrc."""
    h = hashlib.sha256()
    for f in source_files():
        h.update(os.path.basename(f).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()[:16]


def _stamp(src, cmd):
    h = hashlib.sha256(" ".join(cmd[1:]).encode())
    for f in [src] + sorted(glob.glob(os.path.join(HERE, "*.h"))):
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def _compile(src, force, build_dir=None, defines=()):
    obj = os.path.join(build_dir or BUILD, os.path.basename(src).replace(".hip", ".o"))
    cmd = [hipcc()] + _flags(defines) + ["-c", src, "-o", obj]
    stamp = _stamp(src, cmd)
    sfile = obj + ".stamp"
    if not force and os.path.exists(obj) and os.path.exists(sfile):
        with open(sfile) as fh:
            if fh.read().strip() == stamp:
                return obj, False
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
    with open(sfile, "w") as fh:
        fh.write(stamp)
    return obj, True


def _hash_object(build_dir, digest):
    """Object defining ``extern "C" const char* tdq_src_hash()`` (host code)."""
    src = os.path.join(build_dir, "tdq_src_hash.cpp")
    obj = os.path.join(build_dir, "tdq_src_hash.o")
    text = f'extern "C" const char* tdq_src_hash() {{ return "{digest}"; }}\n'
    if os.path.exists(src) and os.path.exists(obj):
        with open(src) as fh:
            if fh.read() == text:
                return obj, False
    with open(src, "w") as fh:
        fh.write(text)
    r = subprocess.run(["g++", "-O2", "-fPIC", "-c", src, "-o", obj], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hash object failed:\n{r.stdout}\n{r.stderr}")
    return obj, True


def build(force=False, jobs=None, verbose=True, variant=None, defines=()):
    """Build ``csrc/libtdq_hip.so``; ``variant="x"`` with ``defines`` builds an A/B variant into
    ``csrc/build_x/libtdq_hip.so`` instead (load it with ``TDQ_LIB_PATH``)."""
    build_dir = os.path.join(HERE, f"build_{variant}") if variant else BUILD
    out = os.path.join(build_dir, "libtdq_hip.so") if variant else OUT
    os.makedirs(build_dir, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(HERE, "*.hip")))
    jobs = jobs or min(len(srcs), max(1, (os.cpu_count() or 2)))
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        results = list(ex.map(lambda s: _compile(s, force, build_dir, defines), srcs))
    hobj, hnew = _hash_object(build_dir, source_hash())
    objs = [o for o, _ in results] + [hobj]
    rebuilt = any(r for _, r in results) or hnew
    if rebuilt or force or not os.path.exists(out) or any(
            os.path.getmtime(o) > os.path.getmtime(out) for o in objs):
        tmp = out + ".tmp"
        # hipRTC: the specialized fused-loss kernels are compiled at run time (csrc/loss_jit.hip)
        cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs + ["-lhiprtc"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, out)
        if verbose:
            print(f"built {out}")
    elif verbose:
        print(f"{out} up to date")
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=None)
    ap.add_argument("--variant", default=None, help="A/B build into csrc/build_<variant>/")
    ap.add_argument("-D", dest="defines", action="append", default=[], help="preprocessor macro (variants)")
    a = ap.parse_args(argv)
    build(force=a.force, jobs=a.j, variant=a.variant, defines=a.defines)


if __name__ == "__main__":
    sys.exit(main())
