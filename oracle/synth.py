"""Seeded synthetic gradients for parity tests and golden fixtures.

TEST INFRASTRUCTURE ONLY. Imported by ``tests/``, ``tests/golden/make_goldens.py``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg. The product path
(``adam-compression_amd/dgc``) never imports anything under ``oracle/``.

The generator is numpy's PCG64 ``standard_normal`` (float32), which is stable for a
fixed numpy (this image and the GPU box share numpy 2.2). Fixtures also store a
digest of every generated input so that a generator drift is caught, not
silently turned into a "parity failure".
"""
import hashlib

import numpy as np

__all__ = ["gradient", "to_bf16_rne", "digest"]


def to_bf16_rne(x):
    """Round float32 values to bfloat16 (round-to-nearest-even), returned as float32.

    This makes the "bf16-origin" inputs of BASELINE.json config 5: many exact
    magnitude ties around the selection threshold.
    """
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return (r & 0xFFFFFFFF).astype(np.uint32).view(np.float32)


def gradient(seed, n, kind="normal", scale=1.0):
    """A float32 gradient of ``n`` elements.

    kind:
      ``normal``  N(0, scale^2)
      ``bf16``    N(0, scale^2) rounded to bf16 (dense ties)
      ``layered`` segments of very different scale (a flat bucket of many layers);
                  the top elements cluster in a few segments
      ``sparse``  90 % exact zeros (+0.0 and -0.0), rest N(0,1)
      ``ties``    small integers (massive ties at every threshold)
    """
    rng = np.random.Generator(np.random.PCG64(seed))
    x = rng.standard_normal(n, dtype=np.float32)
    if scale != 1.0:
        x *= np.float32(scale)
    if kind == "normal":
        pass
    elif kind == "bf16":
        x = to_bf16_rne(x)
    elif kind == "layered":
        seg = max(1, n // 16)
        scales = np.float32(10.0) ** rng.integers(-3, 2, size=(n + seg - 1) // seg).astype(np.float32)
        x *= np.repeat(scales, seg)[:n]
    elif kind == "sparse":
        z = rng.random(n) < 0.9
        x[z] = 0.0
        x[z & (rng.random(n) < 0.5)] = -0.0
    elif kind == "ties":
        x = rng.integers(-8, 9, size=n).astype(np.float32)
    else:
        raise ValueError(f"unknown kind {kind!r}")
    return np.ascontiguousarray(x, dtype=np.float32)


def digest(a):
    """SHA-256 of an array's bytes (dtype and shape are part of the digest)."""
    a = np.ascontiguousarray(a)
    h = hashlib.sha256()
    h.update(str(a.dtype).encode())
    h.update(str(a.shape).encode())
    h.update(a.tobytes())
    return h.hexdigest()
