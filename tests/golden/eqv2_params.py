"""Deterministic EquiformerV2 parameter values for the golden fixtures (test infrastructure).

The fixtures in eqv2.npz were produced by the reference's EquiformerV2_nbody with every
parameter overwritten by ``param_value(name, shape)``; tests rebuild the same state dict from the
recorded key list (eqv2_state.json) without the reference.  Values are O(1) where the reference
initialises them that way and ~1/sqrt(fan_in) for weight matrices, with non-trivial norm affines,
biases and atom-edge embeddings so that every term of the forward is exercised.
"""
from __future__ import annotations

import zlib

import numpy as np


def param_value(name: str, shape) -> np.ndarray:
    shape = tuple(int(s) for s in shape)
    rng = np.random.default_rng(zlib.crc32(name.encode()))
    leaf = name.rsplit(".", 1)[-1]
    if leaf in ("weight",) and len(shape) >= 2:
        if "embedding" in name:                       # nn.Embedding tables
            return 0.5 * rng.standard_normal(shape)
        fan_in = shape[-1]
        return rng.standard_normal(shape) / np.sqrt(fan_in)
    if leaf == "weight" and len(shape) == 1:          # LayerNorm scale
        return 1.0 + 0.2 * rng.standard_normal(shape)
    if leaf == "affine_weight":
        return 1.0 + 0.2 * rng.standard_normal(shape)
    if leaf in ("bias", "affine_bias"):
        return 0.1 * rng.standard_normal(shape)
    if leaf == "alpha_dot":
        return rng.uniform(-1.0, 1.0, shape) / np.sqrt(shape[-1])
    if leaf == "scale":
        return np.full(shape, 1.0)
    return rng.standard_normal(shape)
