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


# ---- the same kernels on caller data (numerics checks against torch fp32 references) --------
def _np(x, dtype):
    import numpy as np
    if hasattr(x, "detach"):             # a torch tensor: host copy, contiguous
        x = x.detach().cpu().contiguous().numpy()
    return np.ascontiguousarray(x, dtype=dtype)


def vector_add_tensors(a, b, device: int = 0):
    """c = a + b with the pod workload's gfx950 vadd kernel; torch in → torch out."""
    import numpy as np
    import torch
    av, bv = _np(a, np.float32).ravel(), _np(b, np.float32).ravel()
    if av.shape != bv.shape:
        raise ValueError(f"shape mismatch {av.shape} vs {bv.shape}")
    return torch.from_numpy(np.asarray(_need().vector_add_arrays(av, bv, device))).reshape(tuple(a.shape))


def mfma_tile(a, b, device: int = 0):
    """C = A @ B on one wave with v_mfma_f32_32x32x16_bf16: A is 32×K, B is K×32 (K a multiple of
    16); inputs are rounded to bf16 as the matrix core sees them, the result is fp32."""
    import numpy as np
    import torch
    a = torch.as_tensor(a).to(torch.bfloat16).contiguous()
    b = torch.as_tensor(b).to(torch.bfloat16).contiguous()
    if a.dim() != 2 or b.dim() != 2 or a.shape[0] != 32 or b.shape[1] != 32 or a.shape[1] != b.shape[0]:
        raise ValueError(f"need A 32xK and B Kx32, got {tuple(a.shape)} and {tuple(b.shape)}")
    k = a.shape[1]
    bits = lambda t: t.view(torch.int16).numpy().view(np.uint16).ravel()   # noqa: E731
    return torch.from_numpy(np.asarray(_need().mfma_tile(bits(a), bits(b), k, device)).copy())


def hbm_pattern(n16: int, seed: int = 0x5EED, device: int = 0):
    """The HBM probe's write pattern for n16 16-byte words, as uint32 words."""
    import numpy as np
    return np.asarray(_need().hbm_pattern(n16, seed, device))


def hbm_verify(words, seed: int = 0x5EED, device: int = 0) -> int:
    """Mismatching 32-bit words of `words` against the probe pattern (the probe's verify kernel)."""
    import numpy as np
    return int(_need().hbm_verify_words(_np(words, np.uint32).ravel(), seed, device))


def hbm_copy(words, device: int = 0):
    import numpy as np
    return np.asarray(_need().hbm_copy_words(_np(words, np.uint32).ravel(), device))
