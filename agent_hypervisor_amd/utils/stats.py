"""Spread batch counters (see ``kStatSpread`` in csrc/include/ahv/hd.h).

Kernels add their per-wave counter sums into one of ``SPREAD`` rows (chosen by
workgroup id) instead of a single address; the launcher folds the rows into
the caller's counter vector afterwards.  Both steps are plain stream-ordered
tensor ops, so they are hipGraph-capturable.
"""

from __future__ import annotations

import torch

SPREAD = 64  # == ahv::kStatSpread


class SpreadCounters:
    def __init__(self, k: int, device) -> None:
        self.buf = torch.zeros((SPREAD, k), dtype=torch.int64, device=device)

    def begin(self) -> torch.Tensor:
        """Zero the rows and return the buffer to pass as the kernel's stats pointer."""
        self.buf.zero_()
        return self.buf

    def add_into(self, stats: torch.Tensor) -> torch.Tensor:
        stats.add_(self.buf.sum(dim=0))
        return stats

    def copy_into(self, stats: torch.Tensor) -> torch.Tensor:
        stats.copy_(self.buf.sum(dim=0))
        return stats
