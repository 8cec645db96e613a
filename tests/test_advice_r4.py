"""Regression tests for the round-4 advisor findings: creation stamps
of non-uuid sessions, checkpoint extras of restored sessions collected out of
order."""

from __future__ import annotations

import types
import uuid

import numpy as np

from agent_hypervisor_amd.models.store import GovernanceStore
from agent_hypervisor_amd.runtime.store_checkpoint import _Collect


def test_non_uuid_stamps_never_look_like_a_uuid4_low_half():
    st = GovernanceStore("cpu", caps={"S": 64, "P": 4, "D": 64, "E": 64, "V": 64, "G": 64, "T": 64, "X": 1 << 16,
                                      "B": 1 << 16})
    try:
        stamps = [st.next_stamp() for _ in range(1000)]
        assert all(s >> 62 == 3 and s != 0 for s in stamps) and len(set(stamps)) == len(stamps)
        for _ in range(1000):  # RFC 4122 variant bits 10 in every uuid4 low half
            lo = int(uuid.uuid4().hex[16:], 16)
            assert lo >> 62 == 2 and lo not in stamps
    finally:
        st.close()


def test_restored_extras_follow_positions_not_sort_order():
    b = types.SimpleNamespace(
        ids=[f"s{i}" for i in range(5)], slots=np.arange(5, dtype=np.int32),
        cfg_mode=np.zeros(5, np.uint8), cfg_maxdur=np.zeros(5), cfg_chain=np.zeros(5, np.uint8),
        dskip=np.zeros(5, np.int32), goff=np.zeros(6, np.int64), delta_off=np.zeros(6, np.int64),
        drows=np.zeros(0, np.int32), extras={4: {"vfs": "four"}, 1: {"vfs": "one"}})
    col = _Collect()
    col.restored(b, np.array([4, 0, 1], dtype=np.int64))  # not ascending
    assert col.ids == ["s4", "s0", "s1"]
    assert col.extras == {0: {"vfs": "four"}, 2: {"vfs": "one"}}


def test_a_row_released_twice_enters_the_free_list_once():
    st = GovernanceStore("cpu", caps={"S": 64, "P": 4, "D": 64, "E": 64, "V": 64, "G": 64, "T": 64, "X": 1 << 16,
                                      "B": 1 << 16})
    try:
        r = st.alloc("S")
        st.release("S", r)
        st.release("S", r)  # a second owner that believed it held the row
        st.release("G", 5)  # never allocated
        assert st.info()["double_releases"] == 2
        st.reclaim()
        rows = [st.alloc("S") for _ in range(64)]
        assert len(set(rows)) == 64  # the row was handed out once
    finally:
        st.close()
