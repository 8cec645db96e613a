"""The in-tree build's staleness check agrees with the build:
right after ``build()`` nothing is stale, and an object newer than the linked
``.so`` (an interrupted build) makes ``needs_build()`` true until ``build()``
relinks."""

from __future__ import annotations

import os
import time

from agent_hypervisor_amd.utils import build as B


def test_needs_build_is_false_right_after_build():
    B.build()
    assert not B.needs_build()
    objs = sorted(B.BUILD.glob("*.o"))
    assert objs
    so = B.ext_path()
    newer = so.stat().st_mtime + 0.001
    os.utime(objs[0], (newer, newer))  # as if compiled after the last link
    try:
        assert B.needs_build()
        time.sleep(0.05)
        B.build()
        assert not B.needs_build()
        assert so.stat().st_mtime >= max(o.stat().st_mtime for o in objs)
    finally:
        B.build()
