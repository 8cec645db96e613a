"""DID transaction-history verification."""

from hypervisor.verification.history import (
    TransactionHistoryVerifier,
    TransactionRecord,
    VerificationResult,
    VerificationStatus,
)

__all__ = ["TransactionHistoryVerifier", "TransactionRecord", "VerificationResult", "VerificationStatus"]
