#!/usr/bin/env python3
"""Record the reference implementation's results for the golden trace.

Runs ``tests/golden_trace.py``'s operation script under the REFERENCE package
(``/root/reference/src``, read-only; imported in a child interpreter whose
``sys.path`` does not contain this repository) with its ``datetime.now`` pinned to
the trace clock and ``uuid.uuid4`` seeded (so a re-recording is identical), and writes one
fixture per seed (``tests/fixtures/reference_trace.json``, ``reference_trace_s7.json``):
``{"seed", "ops", "sids", "results"}``.

    python scripts/gen_reference_trace.py [--check]

``--check`` compares a fresh recording with the committed fixture instead of
writing it (``tests/test_reference_trace.py`` runs this when the reference is
mounted, so the fixture stays pinned to the reference's behaviour).
"""

from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_SRC = "/root/reference/src"
FIXTURES = {  # seed → (fixture, sessions, operations)
    2026: (os.path.join(ROOT, "tests", "fixtures", "reference_trace.json"), 32, 1200),
    7: (os.path.join(ROOT, "tests", "fixtures", "reference_trace_s7.json"), 48, 2400),
}
FIXTURE, SEED = FIXTURES[2026][0], 2026

_CHILD = r"""
import asyncio, datetime as _dt, importlib.util, json, sys
spec = importlib.util.spec_from_file_location("golden_trace", sys.argv[1])
gt = importlib.util.module_from_spec(spec); spec.loader.exec_module(gt)
import random, uuid
_urng = random.Random(int(sys.argv[3]))
uuid.uuid4 = lambda: uuid.UUID(int=_urng.getrandbits(128), version=4)  # reproducible ids across recordings
import hypervisor  # the reference package (only REF_SRC is on sys.path)
assert hypervisor.__file__.startswith(sys.argv[2]), hypervisor.__file__
cur = [gt.BASE_US]
class PinnedDatetime(_dt.datetime):
    @classmethod
    def now(cls, tz=None):
        t = gt.at(cur[0])
        return t if tz is not None else t.replace(tzinfo=None)
    @classmethod
    def utcnow(cls):
        return gt.at(cur[0]).replace(tzinfo=None)
def pin():
    for name, mod in list(sys.modules.items()):
        if name.split(".")[0] == "hypervisor" and getattr(mod, "datetime", None) is _dt.datetime:
            mod.datetime = PinnedDatetime
import pkgutil
for m in pkgutil.walk_packages(hypervisor.__path__, "hypervisor."):
    try:
        importlib.import_module(m.name)
    except Exception:
        pass
pin()
def set_now(us):
    cur[0] = us
seed = int(sys.argv[3])
ops = gt.make_ops(seed, int(sys.argv[4]), int(sys.argv[5]))
out = asyncio.run(gt.run_ops(ops, set_now))
json.dump({"seed": seed, "ops": ops, "sids": out["sids"], "results": out["results"]}, sys.stdout)
"""


def record(seed: int = SEED) -> dict:
    env = {k: v for k, v in os.environ.items() if k not in ("PYTHONPATH",)}
    env.update(PYTHONPATH=REF_SRC, PYTHONDONTWRITEBYTECODE="1")
    _, sessions, nops = FIXTURES[seed]
    p = subprocess.run([sys.executable, "-c", "import importlib; " + _CHILD, os.path.join(ROOT, "tests",
                                                                                          "golden_trace.py"),
                        REF_SRC, str(seed), str(sessions), str(nops)], capture_output=True, text=True, env=env,
                       cwd="/tmp", timeout=600)
    if p.returncode != 0:
        raise RuntimeError(p.stderr[-4000:])
    return json.loads(p.stdout)


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--check", action="store_true")
    args = ap.parse_args()
    bad = 0
    for seed, (fixture, _, _) in FIXTURES.items():
        rec = record(seed)
        if args.check:
            with open(fixture) as f:
                old = json.load(f)
            same = old == json.loads(json.dumps(rec))
            verdict = "matches the reference" if same else "DIFFERS from the reference"
            print(f"{os.path.basename(fixture)}: {verdict}")
            bad += 0 if same else 1
            continue
        os.makedirs(os.path.dirname(fixture), exist_ok=True)
        with open(fixture, "w") as f:
            json.dump(rec, f, separators=(",", ":"))
            f.write("\n")
        errs = sum(1 for r in rec["results"] if "msg" in r)
        print(f"wrote {fixture}: {len(rec['ops'])} ops, {errs} reference errors recorded")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
