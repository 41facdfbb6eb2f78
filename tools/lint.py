"""Minimal static check (flake8 is not installed in this image): the reference CI's
``flake8 --select=E9,F63,F7,F82`` subset (/root/reference/.github/workflows/python-package.yml:31-36)
- E9 / F7: the file must compile (syntax errors, misplaced return / break / continue);
- F63: comparisons against literals with ``is`` / ``is not`` (``x is 1``);
- F82: names read but bound nowhere (module scope, or a global read inside a function).

    python tools/lint.py [paths...]      # default: the package, tests, examples, tools, bench.py
"""
from __future__ import annotations

import ast
import builtins
import os
import sys
import symtable

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEFAULT = ["tensordiffeq_amd", "tensordiffeq", "tests", "examples", "tools", "bench.py", "__graft_entry__.py"]
BUILTINS = set(dir(builtins)) | {"__file__", "__name__", "__doc__", "__spec__", "__builtins__", "__path__",
                                 "__loader__", "__package__", "__annotations__", "__dict__", "__module__",
                                 "__qualname__", "__class__"}


def _files(paths):
    for p in paths:
        p = os.path.join(ROOT, p) if not os.path.isabs(p) else p
        if os.path.isfile(p) and p.endswith(".py"):
            yield p
        elif os.path.isdir(p):
            for d, _, fs in os.walk(p):
                if "__pycache__" in d:
                    continue
                for f in sorted(fs):
                    if f.endswith(".py"):
                        yield os.path.join(d, f)


def _module_bindings(tree):
    names = set()
    for node in ast.walk(tree):
        if isinstance(node, (ast.FunctionDef, ast.AsyncFunctionDef, ast.ClassDef)):
            names.add(node.name)
        elif isinstance(node, ast.Global):
            names.update(node.names)
    top = symtable.symtable(ast.unparse(tree), "<m>", "exec")
    for s in top.get_symbols():
        if s.is_assigned() or s.is_imported() or s.is_namespace():
            names.add(s.get_name())
    return names


def _star(tree):
    return any(isinstance(n, ast.ImportFrom) and any(a.name == "*" for a in n.names) for n in ast.walk(tree))


def check(path):
    errs = []
    src = open(path, encoding="utf-8").read()
    try:
        tree = ast.parse(src, path)
        compile(src, path, "exec")
    except SyntaxError as e:
        return [f"{path}:{e.lineno}: E9 {e.msg}"]
    for node in ast.walk(tree):
        if isinstance(node, ast.Compare):
            for op, rhs in zip(node.ops, node.comparators):
                if isinstance(op, (ast.Is, ast.IsNot)) and isinstance(rhs, ast.Constant) and \
                        not (rhs.value is None or isinstance(rhs.value, bool) or rhs.value is Ellipsis):
                    errs.append(f"{path}:{node.lineno}: F632 use ==/!= to compare with a literal")
    if _star(tree):
        return errs
    bound = _module_bindings(tree) | BUILTINS
    table = symtable.symtable(src, path, "exec")

    def walk(t):
        for s in t.get_symbols():
            n = s.get_name()
            if not s.is_referenced():
                continue
            if t.get_type() == "module":
                if not (s.is_assigned() or s.is_imported() or s.is_namespace()) and n not in bound:
                    errs.append(f"{path}: F821 undefined name {n!r} (module scope)")
            elif s.is_global() and not s.is_declared_global() and n not in bound:
                errs.append(f"{path}: F821 undefined name {n!r} (in {t.get_name()})")
        for c in t.get_children():
            walk(c)
    walk(table)
    return errs


def main(argv=None):
    paths = (argv if argv is not None else sys.argv[1:]) or DEFAULT
    errs = [e for f in _files(paths) for e in check(f)]
    for e in errs:
        print(e)
    print(f"lint: {len(errs)} problem(s)")
    return 1 if errs else 0


if __name__ == "__main__":
    sys.exit(main())
