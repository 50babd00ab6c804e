"""Build the gfx950 kernel library (``_da_kernels.so``) with hipcc — no hipify, no torch headers.

Every ``csrc/*.hip`` file is compiled to an object with ``hipcc --offload-arch=gfx950`` (in
parallel) and linked into one shared library next to this file. The library exports plain
``extern "C"`` launchers (``da_*``) that take raw device pointers and a ``hipStream_t``; Python
binds them with ctypes (``docagents_amd.ops.kernels``), so launches go onto PyTorch's current
HIP stream and are capturable in HIP graphs.

The library links against ``libamdhip64.so.7`` by SONAME; when PyTorch is imported first, the
dynamic loader resolves it to the HIP runtime PyTorch already loaded (one runtime per process).

Usage: ``python -m docagents_amd.ops.build [--force] [--debug]``
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
CSRC = HERE / "csrc"
LIB = HERE / "_da_kernels.so"
LIB_DEBUG = HERE / "_da_kernels_debug.so"  # -O1 -g -DDA_DEBUG: device asserts on (DA_KERNELS_DEBUG=1 loads it)
ARCH = os.environ.get("DA_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found (need ROCm >= 7.0)")


def _sources() -> list[Path]:
    return sorted(CSRC.glob("*.hip"))


def _fingerprint(debug: bool) -> str:
    h = hashlib.sha256()
    for p in sorted(CSRC.glob("*")):
        h.update(p.name.encode())
        h.update(p.read_bytes())
    h.update(f"{ARCH}:{debug}".encode())
    return h.hexdigest()


def _flags(debug: bool) -> list[str]:
    f = [f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-mcode-object-version=5",
         "-Wno-unused-result", "-ffp-contract=fast"]
    f += ["-O1", "-g", "-DDA_DEBUG=1"] if debug else ["-O3"]
    return f


LAST_BUILD: dict = {}


def source_hashes() -> dict:
    """sha256 (first 16 hex) of every kernel source: what a build compiled."""
    return {p.name: hashlib.sha256(p.read_bytes()).hexdigest()[:16] for p in sorted(CSRC.glob("*"))}


def build(force: bool = False, debug: bool = False, verbose: bool = False) -> Path:
    """Compile (if stale) and return the path of the shared library. ``LAST_BUILD`` records what
    happened: mode "compiled" (hipcc ran, with the wall time) or "reused" (fingerprint match)."""
    import time
    lib = LIB_DEBUG if debug else LIB
    stamp = HERE / ("_da_kernels_debug.fingerprint" if debug else "_da_kernels.fingerprint")
    fp = _fingerprint(debug)
    LAST_BUILD.clear()
    LAST_BUILD.update({"lib": str(lib), "fingerprint": fp[:16], "arch": ARCH, "debug": debug})
    if lib.exists() and stamp.exists() and stamp.read_text() == fp and not force:
        LAST_BUILD["mode"] = "reused"
        return lib
    # N ranks of one job import the package at once: one builds, the others wait and reuse it
    import fcntl
    with open(HERE / "_da_kernels.lock", "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        if lib.exists() and stamp.exists() and stamp.read_text() == fp and not force:
            LAST_BUILD["mode"] = "reused"
            return lib
        t0 = time.perf_counter()
        out = _build_locked(stamp, fp, debug, verbose)
        LAST_BUILD.update({"mode": "compiled", "compile_s": round(time.perf_counter() - t0, 1),
                           "sources": source_hashes()})
        return out


def _build_locked(stamp: Path, fp: str, debug: bool, verbose: bool) -> Path:
    hipcc = _hipcc()
    lib = LIB_DEBUG if debug else LIB
    objdir = HERE / ("_build_debug" if debug else "_build")
    objdir.mkdir(exist_ok=True)
    flags = _flags(debug)

    def compile_one(src: Path) -> Path:
        obj = objdir / (src.stem + ".o")
        cmd = [hipcc, *flags, "-c", str(src), "-o", str(obj)]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stderr}")
        return obj

    workers = min(len(_sources()), int(os.environ.get("MAX_JOBS", "8")), 16)
    with cf.ThreadPoolExecutor(max_workers=max(1, workers)) as ex:
        objs = list(ex.map(compile_one, _sources()))
    tmp = lib.with_suffix(f".so.tmp{os.getpid()}")
    cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(tmp)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr}")
    # a kernel whose launch stub the host pass dropped (e.g. a template-dependent array extent in a
    # builtin argument) links fine and fails only at dlopen on the GPU box: catch it here
    nm = shutil.which("nm")
    if nm:
        u = subprocess.run([nm, "-D", "--undefined-only", str(tmp)], capture_output=True, text=True).stdout
        stubs = [ln.split()[-1] for ln in u.splitlines() if "__device_stub__" in ln]
        if stubs:
            tmp.unlink(missing_ok=True)
            raise RuntimeError(f"undefined kernel launch stubs: {stubs[:4]}")
    os.replace(tmp, lib)
    stamp.write_text(fp)
    return lib


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args()
    print(build(force=a.force, debug=a.debug, verbose=a.verbose))


if __name__ == "__main__":
    main()
