"""Reversibility: Execute_API / Undo_API registry."""

from hypervisor.reversibility.registry import ReversibilityEntry, ReversibilityRegistry

__all__ = ["ReversibilityEntry", "ReversibilityRegistry"]
