"""Build and run the host-side AddressSanitizer / UBSan check of the native library
(tools/asan/host_check.cpp): the csrc/*.hip sources with host entry points compiled with
``-Xarch_host -fsanitize=address,undefined`` (device code unsanitized: the pool offers no GPU ASan
/ xnack+), linked with the driver, run on the CPU.  The per-width-class kernel instantiation
tables (jet_bf3_w*.hip: device code only behind a switch) are replaced by stubs in the driver, so
the build takes seconds.  Exit status 0 = clean.

    python tools/asan_host_check.py [-j 8]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(HERE), "tensordiffeq_amd", "csrc")
SAN = ["-Xarch_host", "-fsanitize=address,undefined", "-Xarch_host", "-fno-omit-frame-pointer",
       "-Xarch_host", "-fno-sanitize-recover=all"]


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", type=int, default=min(8, os.cpu_count() or 2))
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    sys.path.insert(0, os.path.dirname(HERE))
    from tensordiffeq_amd.csrc.build import hipcc
    out = a.out or tempfile.mkdtemp(prefix="tdq_asan_")
    os.makedirs(out, exist_ok=True)
    srcs = [f for f in sorted(glob.glob(os.path.join(CSRC, "*.hip"))) if "jet_bf3_w" not in os.path.basename(f)]
    srcs.append(os.path.join(HERE, "asan", "host_check.cpp"))
    base = [hipcc(), "-O1", "-g", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "-I", CSRC] + SAN

    def comp(src):
        obj = os.path.join(out, os.path.basename(src) + ".o")
        lang = ["-x", "hip"] if src.endswith(".cpp") else []
        r = subprocess.run(base + lang + ["-c", src, "-o", obj], capture_output=True, text=True)
        if r.returncode:
            raise RuntimeError(f"{src}:\n{r.stderr[-3000:]}")
        return obj

    with cf.ThreadPoolExecutor(a.j) as ex:
        objs = list(ex.map(comp, srcs))
    exe = os.path.join(out, "host_check")
    r = subprocess.run([hipcc(), "--offload-arch=gfx950", "-fsanitize=address,undefined", "-o", exe] + objs + ["-lhiprtc"],
                       capture_output=True, text=True)
    if r.returncode:
        print(r.stderr[-3000:])
        return 1
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, env=env)
    sys.stdout.write(r.stdout)
    sys.stderr.write(r.stderr[-5000:])
    return r.returncode


if __name__ == "__main__":
    sys.exit(main())
