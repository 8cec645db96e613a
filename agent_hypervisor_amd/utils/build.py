"""In-tree build of the native extension ``agent_hypervisor_amd._C``.

Every source under ``csrc/`` is compiled by ``hipcc --offload-arch=gfx950`` (host
runtime files and HIP kernel files alike) and linked into one shared object placed
next to this package, so the ``.so`` travels with the repository snapshot to the
GPU box.  Object files are cached under ``build/`` and rebuilt only when a source
or any header under ``csrc/include`` changed.

Usage::

    python -m agent_hypervisor_amd.utils.build          # incremental
    python -m agent_hypervisor_amd.utils.build --clean  # from scratch
"""

from __future__ import annotations

import argparse
import fcntl
import os
import shutil
import subprocess
import sys
import sysconfig
import time
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

REPO = Path(__file__).resolve().parents[2]
CSRC = REPO / "csrc"
BUILD = REPO / "build" / "native"
PKG = REPO / "agent_hypervisor_amd"
ARCH = os.environ.get("AHV_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def ext_path() -> Path:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return PKG / f"_C{suffix}"


def _sources() -> list[Path]:
    srcs = (
        sorted((CSRC / "host").glob("*.cpp"))
        + sorted((CSRC / "hip").glob("*.hip"))
        + sorted((CSRC / "cpu").glob("*.cpp"))
    )
    return srcs


def _headers_mtime() -> float:
    newest = Path(__file__).stat().st_mtime  # compiler flags live here
    for h in (CSRC / "include").rglob("*.h"):
        newest = max(newest, h.stat().st_mtime)
    return newest


def _includes() -> list[str]:
    import pybind11

    inc = [
        f"-I{CSRC / 'include'}",
        f"-I{pybind11.get_include()}",
        f"-I{sysconfig.get_paths()['include']}",
        "-I/opt/rocm/include",
    ]
    return inc


def _compile_cmd(src: Path, obj: Path) -> list[str]:
    if src.parent.name == "cpu":
        # host-CPU-only code (x86 intrinsics): plain C++, no offload
        return [
            os.environ.get("CXX", "g++"),
            "-O3",
            "-std=c++17",
            "-fPIC",
            "-fvisibility=hidden",
            f"-I{CSRC / 'include'}",
            "-c",
            str(src),
            "-o",
            str(obj),
        ]
    cmd = [
        HIPCC,
        "-x",
        "hip",
        f"--offload-arch={ARCH}",
        "-O3",
        # Governance arithmetic must round exactly like CPython (no a*b+c fusion):
        # σ_eff, clips, risk and token refills are compared bit-for-bit.
        "-ffp-contract=off",
        "-std=c++17",
        "-fPIC",
        "-fvisibility=hidden",
        "-Wno-unused-result",
        "-Wno-unused-command-line-argument",
        "-DPYBIND11_DETAILED_ERROR_MESSAGES",
        *_includes(),
        "-MMD",
        "-MF",
        str(obj.with_suffix(".d")),
        "-c",
        str(src),
        "-o",
        str(obj),
    ]
    return cmd


def _deps(obj: Path) -> list[Path] | None:
    """Headers an object was compiled from (its -MMD depfile), or None if unknown."""
    d = obj.with_suffix(".d")
    if not d.exists():
        return None
    text = d.read_text().replace("\\\n", " ")
    out = []
    for tok in text.split(":", 1)[-1].split():
        if tok.endswith((".h", ".hpp", ".cuh", ".inc")):
            out.append(Path(tok))
    return out


def _stale(src: Path, obj: Path) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    if src.stat().st_mtime > t or Path(__file__).stat().st_mtime > t:
        return True
    deps = _deps(obj)
    if deps is None:
        return _headers_mtime() > t
    for h in deps:
        try:
            if h.stat().st_mtime > t:
                return True
        except FileNotFoundError:
            return True
    return False


def _link_cmd(objs: list[Path], out: Path) -> list[str]:
    return [
        HIPCC,
        f"--offload-arch={ARCH}",
        "-shared",
        "-fPIC",
        "-o",
        str(out),
        *map(str, objs),
        "-L/opt/rocm/lib",
        "-lamdhip64",
        "-lrccl",
        "-Wl,-rpath,/opt/rocm/lib",
    ]


def needs_build() -> bool:
    out = ext_path()
    if not out.exists():
        return True
    t = out.stat().st_mtime
    if not BUILD.exists():  # fresh checkout with a shipped .so: trust it unless sources are newer
        return _headers_mtime() > t or any(s.stat().st_mtime > t for s in _sources())
    for s in _sources():
        o = BUILD / (s.parent.name + "_" + s.stem + ".o")
        if _stale(s, o) or (o.exists() and o.stat().st_mtime > t):
            return True
    return False


def build(clean: bool = False, jobs: int | None = None, verbose: bool = False) -> Path:
    """Compile and link ``_C``; returns the path of the shared object."""
    BUILD.mkdir(parents=True, exist_ok=True)
    lock_path = BUILD / ".lock"
    with open(lock_path, "w") as lock:
        fcntl.flock(lock, fcntl.LOCK_EX)
        if clean:
            for o in BUILD.glob("*.o"):
                o.unlink()
        srcs = _sources()
        todo: list[tuple[Path, Path]] = []
        objs: list[Path] = []
        for s in srcs:
            o = BUILD / (s.parent.name + "_" + s.stem + ".o")
            objs.append(o)
            if _stale(s, o):
                todo.append((s, o))
        jobs = jobs or min(len(todo) or 1, int(os.environ.get("MAX_JOBS", "8")), 16)
        t0 = time.time()

        def run(pair: tuple[Path, Path]) -> tuple[Path, str]:
            src, obj = pair
            cmd = _compile_cmd(src, obj)
            if verbose:
                print(" ".join(cmd), flush=True)
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr[-8000:]}")
            return src, r.stderr

        if todo:
            with ThreadPoolExecutor(max_workers=jobs) as ex:
                for src, err in ex.map(run, todo):
                    if verbose and err.strip():
                        print(err, file=sys.stderr)
        out = ext_path()
        # relink when anything compiled, the .so is missing, or an object is newer than
        # it (an interrupted earlier build): exactly the objects needs_build() checks
        if todo or not out.exists() or any(o.stat().st_mtime > out.stat().st_mtime for o in objs):
            tmp = out.with_suffix(".tmp.so")
            r = subprocess.run(_link_cmd(objs, tmp), capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"link failed:\n{r.stderr[-8000:]}")
            os.replace(tmp, out)
        if verbose:
            print(f"[ahv build] {len(todo)} compiled, {time.time() - t0:.1f}s -> {out}")
        return out


def main() -> None:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("-v", "--verbose", action="store_true")
    args = ap.parse_args()
    if args.clean and BUILD.exists():
        shutil.rmtree(BUILD)
    build(clean=args.clean, jobs=args.jobs, verbose=True if args.verbose else True)


if __name__ == "__main__":
    main()
