"""The guided demo runs end to end on the CPU host twins (reference C48)."""

from __future__ import annotations

import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_demo_runs_all_sections(capsys):
    spec = importlib.util.spec_from_file_location("ahv_demo", os.path.join(ROOT, "examples", "demo.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    assert mod.main([]) == 0
    out = capsys.readouterr().out
    for needle in ("Session lifecycle", "compensation_failed", "depth=1", "chain ok=False", "critical",
                   "root-match=True"):
        assert needle in out
    assert mod.main(["bogus"]) == 2
