"""Audit: Merkle-chained delta engine, summary-hash commitment, ephemeral GC."""

from hypervisor.audit.commitment import CommitmentEngine, CommitmentRecord
from hypervisor.audit.delta import DeltaEngine, SemanticDelta, VFSChange
from hypervisor.audit.gc import EphemeralGC, GCResult, RetentionPolicy

__all__ = [
    "CommitmentEngine",
    "CommitmentRecord",
    "DeltaEngine",
    "SemanticDelta",
    "VFSChange",
    "EphemeralGC",
    "GCResult",
    "RetentionPolicy",
]
