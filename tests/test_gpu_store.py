"""Device-authoritative store on the MI355X: the public ``Hypervisor`` API with
every state change executed by the resident gfx950 worker.

Independent oracles: host SHA-256 / canonical JSON of the same fields (digests,
records, Merkle roots), and the pure host engines (liability, lifecycle, saga)
for the same call sequence.  The parity suites that re-express the reference's
326 behaviours then run end to end with ``AHV_STORE=cuda``.
"""

from __future__ import annotations

import asyncio

import pytest

from tests.test_store import (
    PARITY_SUITES,
    _run_suites,
    check_lifecycle_errors,
    check_liability_parity,
    check_merkle_roots_track_chain,
    check_pipeline_parity,
    check_saga_compensation,
)

pytestmark = pytest.mark.gpu


def test_pipeline_parity_on_device(cuda_device):
    check_pipeline_parity("cuda")


def test_merkle_roots_track_chain_on_device(cuda_device):
    check_merkle_roots_track_chain("cuda")


def test_liability_parity_on_device(cuda_device):
    check_liability_parity("cuda")


def test_lifecycle_errors_on_device(cuda_device):
    check_lifecycle_errors("cuda")


def test_saga_compensation_on_device(cuda_device):
    check_saga_compensation("cuda")


def test_worker_is_the_executor(cuda_device):
    from hypervisor import Hypervisor

    hv = Hypervisor(device="cuda")
    info = hv._store.info()
    assert info["gpu"] and hv.device == "cuda"


def test_parity_suites_through_device_store(cuda_device):
    _run_suites("cuda", PARITY_SUITES)


@pytest.mark.gpu
def test_captures_never_take_a_torn_slots_arguments():
    """Write-combined slot chunks reach the device in any order; a read that mixes a
    capture's new words with the previous occupant's must be rejected.  The XOR
    checksum let a record-length / hole-offset pair that changed by the same amount
    through (~1 in 3,000 sessions), and the worker hashed the record with another
    capture's length and hole.  Thousands of back-to-back sessions with varying
    record lengths: every device digest equals hashlib over the canonical payload and
    every awaited root equals the host's prediction."""
    import importlib.util
    import os

    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts", "root_stress.py")
    spec = importlib.util.spec_from_file_location("root_stress", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    res = asyncio.run(mod.main(4000, "cuda"))
    assert res["bad_root"] == 0 and res["bad_digest_chains"] == 0, res
