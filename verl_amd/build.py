"""Build libverl_amd.so (the gfx950 HIP kernels + C-ABI) in-tree with hipcc.

The library lands in ``verl_amd/lib/libverl_amd.so`` so that it travels with the repository
snapshot to the GPU box. Objects are compiled in parallel and reused when up to date.

Usage: ``python -m verl_amd.build [--force]``
"""

from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
REPO_DIR = PKG_DIR.parent
CSRC = PKG_DIR / "csrc"
BUILD_DIR = PKG_DIR / "lib" / "obj"
LIB_PATH = PKG_DIR / "lib" / "libverl_amd.so"
HEADERS = [REPO_DIR / "include" / "verl_amd.h", *sorted(CSRC.glob("*.h"))]

ARCH = os.environ.get("VERL_AMD_ARCH", "gfx950")
# -ffp-contract=off: elementwise arithmetic must round like the reference's eager torch ops
# (explicit fmaf() calls are still fused where the kernels ask for them).
CFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-ffp-contract=off", "-Wall"]


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found: the MI355X kernels cannot be built")


def _stale(target: Path, deps: list[Path]) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


# host-only C++ (no device code) is compiled by the system C++ compiler
CXXFLAGS = ["-O2", "-std=c++17", "-fPIC", "-Wall"]


def _compile(hipcc: str, src: Path, obj: Path) -> None:
    if src.suffix == ".cpp":
        cmd = [shutil.which("g++") or "c++", *CXXFLAGS, "-c", str(src), "-o", str(obj)]
    else:
        cmd = [hipcc, *CFLAGS, "-c", str(src), "-o", str(obj)]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"hipcc failed on {src.name}:\n{res.stdout}\n{res.stderr}")


def build(force: bool = False, verbose: bool = False) -> Path:
    hipcc = _hipcc()
    BUILD_DIR.mkdir(parents=True, exist_ok=True)
    sources = sorted(CSRC.glob("*.hip")) + sorted(CSRC.glob("*.cpp"))
    jobs = []
    objs = []
    for src in sources:
        obj = BUILD_DIR / (src.stem + (".o" if src.suffix == ".hip" else ".host.o"))
        objs.append(obj)
        if force or _stale(obj, [src, *HEADERS]):
            jobs.append((src, obj))
    if jobs:
        workers = min(len(jobs), max(1, min(8, os.cpu_count() or 1)))
        with cf.ThreadPoolExecutor(workers) as ex:
            futs = [ex.submit(_compile, hipcc, s, o) for s, o in jobs]
            for f in futs:
                f.result()
        if verbose:
            print(f"[verl_amd.build] compiled {len(jobs)} source(s) for {ARCH}")
    if force or jobs or _stale(LIB_PATH, objs):
        cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(LIB_PATH), *map(str, objs)]
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"link failed:\n{res.stdout}\n{res.stderr}")
        if verbose:
            print(f"[verl_amd.build] linked {LIB_PATH}")
    return LIB_PATH


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    args = ap.parse_args(argv)
    build(force=args.force, verbose=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
