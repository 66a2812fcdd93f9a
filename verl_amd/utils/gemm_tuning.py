"""Tuned hipBLASLt / rocBLAS solution tables for the model GEMMs (q|k|v, o, gate|up, down).

hipBLASLt's default heuristic picks poorly for the actor's skinny shapes on gfx950 (H = 896
outputs, tens of thousands of packed tokens): an exhaustive search over the hipBLASLt and rocBLAS
solutions finds 1.1-1.4x faster kernels (tools/tunableop_probe.py at 690aed1, profiles/r01/). The search is
too slow to run inside a training job, so it runs once offline (tools/tune_gemms.py) over the
shapes a workload produces and the winners are committed as a table under
``verl_amd/tuned/``. At run time PyTorch's TunableOp dispatcher looks every GEMM up in that table
(tuning disabled, nothing written back); a shape that is not in the table keeps the default
heuristic. The tables key on exact (M, N, K), which is why the actor rounds packed micro-batches
up to a multiple of ``pack_pad_multiple`` tokens (dp_actor._plan_packing).

The table's validator lines pin the PyTorch, HIP, hipBLASLt and rocBLAS versions and the gfx arch;
TunableOp ignores a table that does not match the running stack.
"""

from __future__ import annotations

import os

import torch

TUNED_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tuned")
DEFAULT_TABLE = os.path.join(TUNED_DIR, "gemm_qwen2_0p5b_mi355x.csv")

_loaded: str | None = None
_shapes: frozenset = frozenset()  # "nt_M_N_K" problem prefixes present in the loaded table


def resolve(path: str) -> str:
    if path in ("default", True):
        return DEFAULT_TABLE
    if not os.path.isabs(path) and not os.path.exists(path):
        cand = os.path.join(TUNED_DIR, path)
        if os.path.exists(cand):
            return cand
    return path


def use_tuned_gemms(path: str = "default") -> bool:
    """Route torch GEMMs through TunableOp with the solution table at ``path`` (lookup only).
    Returns False (and leaves the default heuristic in place) when the table is missing or no GPU
    is present."""
    global _loaded
    path = resolve(path)
    if _loaded == path:
        return True
    if not torch.cuda.is_available() or not os.path.exists(path):
        return False
    tun = torch.cuda.tunable
    tun.enable(True)
    tun.tuning_enable(False)
    ok = tun.read_file(path)
    if not ok:
        tun.enable(False)
        return False
    # anything TunableOp writes back at exit goes to a per-process scratch file, never the table
    # (concurrent ranks share it)
    tun.set_filename(os.path.join("/tmp", f"verl_amd_tunableop_{os.getpid()}.csv"), False)
    _loaded = path
    global _shapes
    _shapes = frozenset("_".join(line.split(",")[1].split("_")[:4]) for line in open(path)
                        if line.startswith("Gemm"))
    return True


def has_tuned(op: str, m: int, n: int, k: int) -> bool:
    """Whether the loaded table holds a solution for this BLAS problem (``op`` as TunableOp writes
    it: "nn", "nt", "tn", "tt"; column-major m, n, k)."""
    return f"{op}_{m}_{n}_{k}" in _shapes


def start_tuning(path: str, max_iterations: int = 10, max_duration_ms: int = 30) -> None:
    """Offline tuning mode (tools/tune_gemms.py): every new GEMM shape is searched and appended to
    ``path``."""
    tun = torch.cuda.tunable
    tun.enable(True)
    tun.tuning_enable(True)
    tun.set_max_tuning_iterations(max_iterations)
    tun.set_max_tuning_duration(max_duration_ms)
    tun.set_filename(path, False)
    if os.path.exists(path):
        tun.read_file(path)


def finish_tuning() -> None:
    torch.cuda.synchronize()
    torch.cuda.tunable.tuning_enable(False)
