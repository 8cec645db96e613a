"""Execution rings: enforcement, classification, elevation, breach detection."""

from hypervisor.rings.breach_detector import BreachEvent, BreachSeverity, RingBreachDetector
from hypervisor.rings.elevation import RingElevation, RingElevationError, RingElevationManager

__all__ = [
    "RingElevationManager",
    "RingElevation",
    "RingElevationError",
    "RingBreachDetector",
    "BreachEvent",
    "BreachSeverity",
]
