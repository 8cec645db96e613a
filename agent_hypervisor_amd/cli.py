"""Console entry points (``ahv-serve``, ``ahv-bench``)."""

from __future__ import annotations

import argparse
import os
import runpy
import sys

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def serve_main(argv=None) -> int:
    """Serve the REST API (hypervisor.api.server:app) with uvicorn."""
    ap = argparse.ArgumentParser(prog="ahv-serve", description=serve_main.__doc__)
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=8000)
    ap.add_argument("--log-level", default="info")
    args = ap.parse_args(argv)
    import uvicorn

    uvicorn.run("hypervisor.api.server:app", host=args.host, port=args.port, log_level=args.log_level)
    return 0


def bench_main(argv=None) -> int:
    """Run the headline benchmark (bench.py at the repository root)."""
    path = os.path.join(_ROOT, "bench.py")
    if not os.path.exists(path):
        print("ahv-bench needs a source checkout (bench.py not found)", file=sys.stderr)
        return 2
    sys.argv = [path, *(argv if argv is not None else sys.argv[1:])]
    runpy.run_path(path, run_name="__main__")
    return 0
