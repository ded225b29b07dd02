"""In-process HIP validation kernels (amdkube._native._hipops, built from native/hipops.hip
and kernels/gpu_common.h for gfx950). Importing this module on a machine with /dev/kfd but
without the built extension raises — GPU code paths never fall back silently."""
from __future__ import annotations

import os

try:
    from .._native import _hipops as _ext  # type: ignore
except ImportError as e:
    _ext = None
    _err = e
    if os.path.exists("/dev/kfd") or os.environ.get("AMDKUBE_REQUIRE_NATIVE") == "1":
        raise ImportError(f"amdkube HIP extension _hipops not built (python native/build.py): {e}")


def _need():
    if _ext is None:
        raise RuntimeError(f"HIP extension unavailable: {_err}")
    return _ext


def device_count() -> int:
    return _need().device_count()


def device_info(device: int = 0) -> dict:
    return _need().device_info(device)


def vector_add(n: int = 50000, device: int = 0) -> dict:
    return _need().vector_add(n, device)


def hbm_probe(mib: int = 1024, iters: int = 5, device: int = 0) -> dict:
    return _need().hbm_probe(mib, iters, device)


def mfma_burn(ms: float = 100.0, device: int = 0) -> dict:
    return _need().mfma_burn(ms, device)
