"""Build the HIP library of a git revision into ``csrc/build_<name>/libtdq_hip.so`` (A/B baseline).

    python tools/build_ref_lib.py [--rev HEAD] [--name prev]

The sources of that revision are exported with ``git show`` (the working tree is untouched); load
the result with ``TDQ_LIB_PATH=.../csrc/build_<name>/libtdq_hip.so`` next to the current library.
"""
import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rev", default="HEAD")
    ap.add_argument("--name", default="prev")
    a = ap.parse_args()
    from tensordiffeq_amd.csrc import build as B
    out = os.path.join(ROOT, "tensordiffeq_amd", "csrc", f"build_{a.name}")
    src = os.path.join(out, "src")
    shutil.rmtree(out, ignore_errors=True)
    os.makedirs(src)
    files = subprocess.run(["git", "ls-files", "tensordiffeq_amd/csrc"], cwd=ROOT, capture_output=True, text=True,
                           check=True).stdout.split()
    for f in files:
        if f.endswith((".hip", ".h")):
            blob = subprocess.run(["git", "show", f"{a.rev}:{f}"], cwd=ROOT, capture_output=True, check=True).stdout
            with open(os.path.join(src, os.path.basename(f)), "wb") as fh:
                fh.write(blob)
    flags = [f for f in B._flags() if f != B.HERE and f != "-I"] + ["-I", src]

    def comp(s):
        o = os.path.join(out, os.path.basename(s).replace(".hip", ".o"))
        r = subprocess.run([B.hipcc()] + flags + ["-c", s, "-o", o], capture_output=True, text=True)
        if r.returncode:
            raise RuntimeError(r.stderr[-2000:])
        return o

    with cf.ThreadPoolExecutor(8) as ex:
        objs = list(ex.map(comp, sorted(glob.glob(os.path.join(src, "*.hip")))))
    lib = os.path.join(out, "libtdq_hip.so")
    subprocess.run([B.hipcc(), f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", lib] + objs + ["-lhiprtc"],
                   check=True)
    for o in objs:
        os.remove(o)
    shutil.rmtree(src)
    print(lib)


if __name__ == "__main__":
    main()
