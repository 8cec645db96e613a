"""Security: per-agent rate limiting and the kill switch."""

from hypervisor.security.kill_switch import KillResult, KillSwitch
from hypervisor.security.rate_limiter import AgentRateLimiter, RateLimitExceeded

__all__ = ["AgentRateLimiter", "RateLimitExceeded", "KillSwitch", "KillResult"]
