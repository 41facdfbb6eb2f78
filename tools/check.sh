#!/bin/bash
# CI-style check (mirrors the reference's GitHub Actions job, .github/workflows/python-package.yml:
# lint subset + import smoke), plus what this repo adds: the gfx950 build of every HIP source, its
# source-hash stamp, and the CPU test suite.  GPU tiers run separately (pytest -m gpu on MI355X).
set -euo pipefail
cd "$(dirname "$0")/.."
python tools/lint.py
python -c "import __graft_entry__ as g; g.build()"
python -c "import tensordiffeq_amd as tdq, tensordiffeq; from tensordiffeq_amd.ops import _lib; \
lib = _lib.load(); assert _lib.library_hash(lib) == _lib.expected_hash(); print('import ok', tdq.__name__)"
python tools/asan_host_check.py   # host-side ASan + UBSan of the native library (~2.5 min)
python -m pytest tests -x -q -m "not gpu"
