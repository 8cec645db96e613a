"""Spread batch counters (see ``kStatSpread`` in csrc/include/ahv/hd.h).

Kernels add their per-wave counter sums into one of ``SPREAD`` rows (chosen by
workgroup id) instead of a single address; the launcher folds the rows into
the caller's counter vector afterwards.  Both steps are stream-ordered, so they
are hipGraph-capturable.

On the device the fold is one single-wave kernel (``spread_fold_kernel`` in
csrc/hip/pipeline.hip) that sums the rows, adds or copies them into the caller's
vector and re-zeroes them: the rows stay zero between launches, so ``begin`` is
free and a batch costs one extra launch instead of three (fill, reduce, add).
"""

from __future__ import annotations

import torch

from agent_hypervisor_amd._native import C

SPREAD = 64  # == ahv::kStatSpread


class SpreadCounters:
    def __init__(self, k: int, device) -> None:
        self.buf = torch.zeros((SPREAD, k), dtype=torch.int64, device=device)

        self.k = k

    def begin(self) -> torch.Tensor:
        """Return the zeroed rows to pass as the kernel's stats pointer."""
        if not self.buf.is_cuda:  # the device fold leaves them zeroed
            self.buf.zero_()
        return self.buf

    def _fold(self, stats: torch.Tensor, accumulate: bool) -> bool:
        if not (self.buf.is_cuda and stats.device == self.buf.device and stats.dtype == torch.int64
                and stats.is_contiguous() and stats.numel() == self.k):
            return False
        stream = torch.cuda.current_stream(self.buf.device).cuda_stream
        C.spread_fold(self.buf.data_ptr(), stats.data_ptr(), self.k, accumulate, stream)
        return True

    def add_into(self, stats: torch.Tensor) -> torch.Tensor:
        if not self._fold(stats, True):
            stats.add_(self.buf.sum(dim=0))
            self.buf.zero_()
        return stats

    def copy_into(self, stats: torch.Tensor) -> torch.Tensor:
        if not self._fold(stats, False):
            stats.copy_(self.buf.sum(dim=0))
            self.buf.zero_()
        return stats
