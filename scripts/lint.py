#!/usr/bin/env python3
"""Self-contained static checks for the Python tree (no third-party linter needed).

The CI lint job runs ruff + mypy (``.github/workflows/ci.yml``) where they can be
installed; this script checks the subset of those rules that matters most and that
the standard library can decide exactly, so the check also runs — and is seen to
pass — in environments without them (``tests/test_lint.py`` runs it on every CPU
test pass):

* E999  every file compiles (``compile(..., "exec")``);
* F401  imported names that are never used (``__init__`` re-exports, ``__all__``
        and ``# noqa`` lines exempt);
* F541  f-strings without a placeholder;
* F632  ``is`` / ``is not`` against a str / bytes / int literal;
* E711 / E712  ``==`` / ``!=`` against ``None`` / ``True`` / ``False``;
* B006  mutable default arguments (list / dict / set displays);
* E501  code lines longer than ``[tool.ruff] line-length`` (120; lines inside multi-line
        string literals — embedded HTML / JS — are exempt);
* W291 / W293  trailing whitespace.

    python scripts/lint.py [paths...]      # exit 1 and one line per finding
"""

from __future__ import annotations

import ast
import os
import sys
import tokenize

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEFAULT_PATHS = ["hypervisor", "agent_hypervisor_amd", "tests", "benchmarks", "examples", "scripts", "bench.py",
                 "__graft_entry__.py", "setup.py"]
LINE_LENGTH = 120


def _noqa_lines(src: str) -> set:
    out = set()
    for i, line in enumerate(src.splitlines(), 1):
        if "# noqa" in line:
            out.add(i)
    return out


class _Uses(ast.NodeVisitor):
    """Every name read anywhere in a module (loads, attribute roots, __all__ strings)."""

    def __init__(self) -> None:
        self.names: set = set()

    def visit_Name(self, node: ast.Name) -> None:
        self.names.add(node.id)

    def visit_Attribute(self, node: ast.Attribute) -> None:
        self.generic_visit(node)

    def visit_Constant(self, node: ast.Constant) -> None:
        # names mentioned in string annotations ("Foo", "Optional[Bar]")
        if isinstance(node.value, str) and node.value.isidentifier():
            self.names.add(node.value)


def _all_names(tree: ast.Module) -> set:
    out = set()
    for node in tree.body:
        if isinstance(node, (ast.Assign, ast.AugAssign)):
            targets = node.targets if isinstance(node, ast.Assign) else [node.target]
            if any(isinstance(t, ast.Name) and t.id == "__all__" for t in targets):
                for elt in getattr(node.value, "elts", []):
                    if isinstance(elt, ast.Constant) and isinstance(elt.value, str):
                        out.add(elt.value)
    return out


def _string_annotation_names(tree: ast.Module) -> set:
    """Identifiers inside string annotations (``-> "DeviceSession"``, ``x: "Optional[Foo]"``)."""
    out = set()
    for node in ast.walk(tree):
        ann = []
        if isinstance(node, (ast.FunctionDef, ast.AsyncFunctionDef)):
            ann.append(node.returns)
            for a in node.args.args + node.args.kwonlyargs + node.args.posonlyargs:
                ann.append(a.annotation)
            for a in (node.args.vararg, node.args.kwarg):
                if a is not None:
                    ann.append(a.annotation)
        elif isinstance(node, ast.AnnAssign):
            ann.append(node.annotation)
        for a in ann:
            if isinstance(a, ast.Constant) and isinstance(a.value, str):
                try:
                    sub = ast.parse(a.value, mode="eval")
                except SyntaxError:
                    continue
                out.update(n.id for n in ast.walk(sub) if isinstance(n, ast.Name))
    return out


def check_file(path: str) -> list[str]:
    with open(path, "rb") as f:
        raw = f.read()
    try:
        src = raw.decode("utf-8")
    except UnicodeDecodeError as e:
        return [f"{path}:1: E902 not UTF-8: {e}"]
    out = []
    try:
        tree = ast.parse(src, filename=path)
        compile(src, path, "exec")
    except SyntaxError as e:
        return [f"{path}:{e.lineno}: E999 {e.msg}"]
    noqa = _noqa_lines(src)
    # ---- F401: unused imports
    uses = _Uses()
    uses.visit(tree)
    used = uses.names | _all_names(tree) | _string_annotation_names(tree)
    is_init = os.path.basename(path) == "__init__.py"
    for node in ast.walk(tree):
        if not isinstance(node, (ast.Import, ast.ImportFrom)) or node.lineno in noqa:
            continue
        if isinstance(node, ast.ImportFrom) and node.module == "__future__":
            continue
        for alias in node.names:
            if alias.name == "*":
                continue
            bound = alias.asname or alias.name.split(".")[0]
            if bound in used:
                continue
            if is_init and node in tree.body:  # a package's public re-exports
                continue
            if alias.asname and alias.asname == alias.name:  # explicit re-export (`import x as x`)
                continue
            out.append(f"{path}:{node.lineno}: F401 '{alias.name}' imported but unused")
    # ---- expression-level rules
    specs = {id(n.format_spec) for n in ast.walk(tree) if isinstance(n, ast.FormattedValue) and n.format_spec}
    for node in ast.walk(tree):
        ln = getattr(node, "lineno", 0)
        if ln in noqa:
            continue
        if isinstance(node, ast.JoinedStr) and id(node) not in specs \
                and not any(isinstance(v, ast.FormattedValue) for v in node.values):
            out.append(f"{path}:{ln}: F541 f-string without any placeholders")
        elif isinstance(node, ast.Compare):
            left = node.left
            for op, right in zip(node.ops, node.comparators):
                if isinstance(op, (ast.Is, ast.IsNot)):
                    for side in (left, right):
                        if isinstance(side, ast.Constant) and isinstance(side.value, (str, bytes, int)) \
                                and not isinstance(side.value, bool):
                            out.append(f"{path}:{ln}: F632 use ==/!= to compare constant literals")
                if isinstance(op, (ast.Eq, ast.NotEq)):
                    for side in (left, right):
                        if isinstance(side, ast.Constant) and side.value is None:
                            out.append(f"{path}:{ln}: E711 comparison to None should be 'is' / 'is not'")
                        elif isinstance(side, ast.Constant) and isinstance(side.value, bool):
                            out.append(f"{path}:{ln}: E712 comparison to {side.value} should be 'is' / truth test")
                left = right
        elif isinstance(node, (ast.FunctionDef, ast.AsyncFunctionDef, ast.Lambda)):
            for d in node.args.defaults + [d for d in node.args.kw_defaults if d is not None]:
                if isinstance(d, (ast.List, ast.Dict, ast.Set)):
                    out.append(f"{path}:{d.lineno}: B006 mutable default argument")
    # ---- physical lines
    try:
        toks = list(tokenize.generate_tokens(iter(src.splitlines(keepends=True)).__next__))
    except (tokenize.TokenError, SyntaxError):
        toks = []
    in_string = set()
    for t in toks:  # lines inside multi-line strings keep their trailing whitespace rules (W291 applies to code only)
        if t.type == tokenize.STRING and t.start[0] != t.end[0]:
            in_string.update(range(t.start[0] + 1, t.end[0] + 1))
    for i, line in enumerate(src.splitlines(), 1):
        if i in noqa:
            continue
        if len(line) > LINE_LENGTH and i not in in_string:  # (embedded HTML / JS text is data)
            out.append(f"{path}:{i}: E501 line too long ({len(line)} > {LINE_LENGTH})")
        if line != line.rstrip() and i not in in_string:
            out.append(f"{path}:{i}: {'W293' if not line.strip() else 'W291'} trailing whitespace")
    return out


def iter_files(paths: list[str]):
    for p in paths:
        p = os.path.join(ROOT, p) if not os.path.isabs(p) else p
        if os.path.isfile(p) and p.endswith(".py"):
            yield p
        elif os.path.isdir(p):
            for d, dirs, files in os.walk(p):
                dirs[:] = sorted(x for x in dirs if x not in ("__pycache__", "build", "fixtures", "gpurun_out"))
                for f in sorted(files):
                    if f.endswith(".py"):
                        yield os.path.join(d, f)


def main(argv: list[str]) -> int:
    findings = []
    n = 0
    for f in iter_files(argv or DEFAULT_PATHS):
        n += 1
        findings.extend(check_file(f))
    for line in findings:
        print(os.path.relpath(line, ROOT) if line.startswith(ROOT) else line)
    print(f"lint: {n} files, {len(findings)} findings", file=sys.stderr)
    return 1 if findings else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
