"""Integration adapters to external Agent-OS services.

* :mod:`~hypervisor.integrations.nexus_adapter` — trust scoring → σ / ring;
* :mod:`~hypervisor.integrations.cmvk_adapter` — behavioural drift → slashing;
* :mod:`~hypervisor.integrations.iatp_adapter` — capability manifests → actions.

Each service is reached through a ``typing.Protocol`` (duck typing), so no
external package is required.
"""
