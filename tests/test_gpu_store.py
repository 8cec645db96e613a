"""Device-authoritative store on the MI355X: the public ``Hypervisor`` API with
every state change executed by the resident gfx950 worker.

Independent oracles: host SHA-256 / canonical JSON of the same fields (digests,
records, Merkle roots), and the pure host engines (liability, lifecycle, saga)
for the same call sequence.  The parity suites that re-express the reference's
326 behaviours then run end to end with ``AHV_STORE=cuda``.
"""

from __future__ import annotations

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
