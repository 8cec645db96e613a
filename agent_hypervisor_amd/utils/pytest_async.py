"""Minimal pytest plugin that runs ``async def`` tests (pytest-asyncio is not
installed in this image).  Registered from ``tests/conftest.py`` and usable as
``-p agent_hypervisor_amd.utils.pytest_async`` for other suites.

Async fixtures are not needed by any suite here; coroutine test functions are
executed with ``asyncio.run`` in a fresh event loop.
"""

from __future__ import annotations

import asyncio
import inspect

import pytest


def pytest_configure(config):
    config.addinivalue_line("markers", "asyncio: run the coroutine test in an event loop")


@pytest.hookimpl(tryfirst=True)
def pytest_pyfunc_call(pyfuncitem):
    fn = pyfuncitem.obj
    if inspect.iscoroutinefunction(fn):
        names = pyfuncitem._fixtureinfo.argnames
        kwargs = {n: pyfuncitem.funcargs[n] for n in names}
        asyncio.run(fn(**kwargs))
        return True
    return None
