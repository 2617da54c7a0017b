"""Deterministic, platform-independent test values (no RNG state, no stored weights).

Used by ``gen_fixtures.py`` (which feeds them to the imported reference) and by the
tests (which feed them to the oracle and the HIP product path), so that committed
fixtures only hold outputs, never multi-MB weight dumps.
"""
from __future__ import annotations

import numpy as np
import torch

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def hash_uniform(n: int, seed: int) -> np.ndarray:
    """splitmix64 of (index, seed) -> float64 uniform in [-0.5, 0.5). Exact integer math."""
    with np.errstate(over="ignore"):
        z = np.arange(n, dtype=np.uint64) + np.uint64(seed) * np.uint64(0x9E3779B97F4A7C15)
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return (z >> np.uint64(11)).astype(np.float64) / float(1 << 53) - 0.5


def tensor(shape, seed: int, scale: float = 1.0, offset: float = 0.0) -> torch.Tensor:
    n = int(np.prod(shape)) if len(shape) else 1
    v = hash_uniform(n, seed) * 2.0 * scale + offset
    return torch.from_numpy(v.astype(np.float32).reshape(shape))


def fill_state(module: torch.nn.Module, seed: int = 1234) -> None:
    """Overwrite every float parameter and BN buffer of a (reference-structured) module
    with deterministic values. Integer index parameters (``shift_in``/``shift_out`` of
    ``Shift_gcn``) are left untouched (they are computed, not learned)."""
    with torch.no_grad():
        items = list(module.named_parameters()) + list(module.named_buffers())
        for k, (name, p) in enumerate(sorted(items, key=lambda kv: kv[0])):
            if not p.dtype.is_floating_point:
                continue
            s = seed + 7919 * (k + 1)
            leaf = name.rsplit(".", 1)[-1]
            shape = tuple(p.shape)
            if leaf == "xpos":
                v = tensor(shape, s, 1e-8)
            elif leaf == "ypos":
                v = tensor(shape, s, 2.0)          # fractional, both signs, |y| up to 2
            elif leaf == "running_mean":
                v = tensor(shape, s, 0.05)
            elif leaf == "running_var":
                v = tensor(shape, s, 0.2, 1.0)
            elif leaf == "num_batches_tracked":
                continue
            elif leaf == "weight" and p.dim() == 1:          # every 1-D weight is a BN gamma
                v = tensor(shape, s, 0.2, 1.0)
            elif leaf in ("bias", "Linear_bias"):
                v = tensor(shape, s, 0.1)
            elif leaf == "Feature_Mask":
                v = tensor(shape, s, 0.5)
            elif leaf == "Linear_weight":
                v = tensor(shape, s, float(np.sqrt(3.0 / shape[0])))
            elif p.dim() >= 2:
                fan_in = int(np.prod(shape[1:]))
                v = tensor(shape, s, float(np.sqrt(3.0 / fan_in)))
            else:
                v = tensor(shape, s, 0.1)
            p.copy_(v.to(p.dtype))
