"""REST front-end of the hypervisor (FastAPI); ``create_app()`` builds the app."""

from hypervisor.api.server import create_app

__all__ = ["create_app"]
