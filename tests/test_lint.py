"""The repository passes its own static checks (``scripts/lint.py``: compile, unused
imports, f-strings without placeholders, literal identity / None / bool comparisons,
mutable defaults, line length, trailing whitespace) — the subset of the CI ruff rules
the standard library decides, so the check runs wherever the tests run."""

import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_static_checks_pass():
    p = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "lint.py")], capture_output=True, text=True,
                       timeout=300, cwd=ROOT)
    assert p.returncode == 0, p.stdout[-4000:] + p.stderr[-1000:]


def test_lint_finds_what_it_checks(tmp_path):
    bad = tmp_path / "bad.py"
    bad.write_text("import os\nx = f'plain'\nif x == None:\n    pass\ndef f(a=[]):\n    return a \n")
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    try:
        import lint
    finally:
        sys.path.pop(0)
    codes = sorted(line.split()[1] for line in lint.check_file(str(bad)))
    assert codes == ["B006", "E711", "F401", "F541", "W291"]
