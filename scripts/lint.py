"""Stdlib-only lint for this repo (the reference's `.lintrunner.toml:5-89` linters, minus the
third-party tools this image does not ship: black / flake8 / mypy / bandit are not importable).

Checks, per file:
  * Python: compiles; no trailing whitespace; no tabs; lines <= 110 columns; final newline;
    no unused top-level imports (``ast`` name scan, ``__init__`` re-exports and ``noqa`` excepted);
    no bare ``except:``.
  * C++ / HIP (``csrc/``, ``research/lab``): no trailing whitespace; no tabs; final newline;
    lines <= 150 columns (long MFMA intrinsics).

    python scripts/lint.py            # lint the tree, exit 1 on findings
    python scripts/lint.py FILE...    # lint given files
"""

from __future__ import annotations

import ast
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PY_DIRS = ["ddlb_amd", "tests", "scripts", "research/diag", "."]
CXX_DIRS = ["csrc", "research/lab"]
CXX_EXT = (".hip", ".cpp", ".h", ".hpp")
SKIP_DIRS = {".git", "build", "gpurun_out", "__pycache__", "results", "profiles"}
PY_MAX = 110
CXX_MAX = 150


def _walk(top: str, exts, recurse: bool = True):
    top = os.path.join(ROOT, top)
    if not recurse:
        for f in sorted(os.listdir(top)):
            if f.endswith(exts) and os.path.isfile(os.path.join(top, f)):
                yield os.path.join(top, f)
        return
    for dirpath, dirnames, files in os.walk(top):
        dirnames[:] = sorted(d for d in dirnames if d not in SKIP_DIRS)
        for f in sorted(files):
            if f.endswith(exts):
                yield os.path.join(dirpath, f)


def _text_checks(path: str, text: str, max_len: int, out: list) -> None:
    rel = os.path.relpath(path, ROOT)
    if text and not text.endswith("\n"):
        out.append(f"{rel}: missing final newline")
    for i, line in enumerate(text.splitlines(), 1):
        if line != line.rstrip():
            out.append(f"{rel}:{i}: trailing whitespace")
        if "\t" in line:
            out.append(f"{rel}:{i}: tab character")
        if len(line) > max_len and "noqa" not in line and "http" not in line:
            out.append(f"{rel}:{i}: line too long ({len(line)} > {max_len})")


def _unused_imports(tree: ast.Module, text: str) -> list:
    imported = {}
    for node in tree.body:
        if isinstance(node, (ast.Import, ast.ImportFrom)):
            if isinstance(node, ast.ImportFrom) and node.module == "__future__":
                continue
            for a in node.names:
                name = (a.asname or a.name).split(".")[0]
                if name != "*":
                    imported[name] = node.lineno
    if not imported:
        return []
    used = set()
    for node in ast.walk(tree):
        if isinstance(node, ast.Name):
            used.add(node.id)
        elif isinstance(node, ast.Attribute):
            base = node
            while isinstance(base, ast.Attribute):
                base = base.value
            if isinstance(base, ast.Name):
                used.add(base.id)
    exported = set()
    for node in tree.body:  # names listed in __all__ count as used
        if isinstance(node, ast.Assign) and any(
                isinstance(t, ast.Name) and t.id == "__all__" for t in node.targets):
            if isinstance(node.value, (ast.List, ast.Tuple)):
                exported |= {e.value for e in node.value.elts if isinstance(e, ast.Constant)}
    lines = text.splitlines()
    return [(n, ln) for n, ln in imported.items()
            if n not in used and n not in exported and "noqa" not in lines[ln - 1]
            and f"'{n}'" not in text and f'"{n}"' not in text]


def lint_py(path: str, out: list) -> None:
    rel = os.path.relpath(path, ROOT)
    with open(path, encoding="utf-8") as f:
        text = f.read()
    _text_checks(path, text, PY_MAX, out)
    try:
        tree = ast.parse(text, filename=path)
    except SyntaxError as e:
        out.append(f"{rel}:{e.lineno}: syntax error: {e.msg}")
        return
    for node in ast.walk(tree):
        if isinstance(node, ast.ExceptHandler) and node.type is None:
            out.append(f"{rel}:{node.lineno}: bare except")
    if os.path.basename(path) != "__init__.py":
        for name, ln in _unused_imports(tree, text):
            out.append(f"{rel}:{ln}: unused import '{name}'")


def lint_cxx(path: str, out: list) -> None:
    with open(path, encoding="utf-8", errors="replace") as f:
        _text_checks(path, f.read(), CXX_MAX, out)


def collect():
    py, cxx = [], []
    for d in PY_DIRS:
        py += list(_walk(d, (".py",), recurse=(d != ".")))
    for d in CXX_DIRS:
        if os.path.isdir(os.path.join(ROOT, d)):
            cxx += list(_walk(d, CXX_EXT))
    return sorted(set(py)), sorted(set(cxx))


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    if argv:
        py = [os.path.abspath(a) for a in argv if a.endswith(".py")]
        cxx = [os.path.abspath(a) for a in argv if a.endswith(CXX_EXT)]
    else:
        py, cxx = collect()
    out: list = []
    for p in py:
        lint_py(p, out)
    for p in cxx:
        lint_cxx(p, out)
    for line in out:
        print(line)
    print(f"lint: {len(py)} python + {len(cxx)} c++/hip files, {len(out)} finding(s)")
    return 1 if out else 0


if __name__ == "__main__":
    sys.exit(main())
