"""Deterministic parameter/input recipe shared by the fixture generator and the tests.

Parameters are NOT stored in the fixtures: both the reference module (at generation time) and
the build's module (at test time) are filled from the same recipe over their state_dict keys
(SURVEY §8c item 7), which also proves the two state_dicts have identical keys and shapes.

  * float parameter `key`: default_rng(crc32(key)).standard_normal(shape) * 0.05
  * LayerNorm weight:      1 + 0.1 * N(0,1)  (so zero-initialised res-post-norms are live)
  * logit_scale:           left at log(10) (swin_v2_module.py:87)
Inputs: default_rng(seed).standard_normal(shape) as float32.
"""
import zlib

import numpy as np
import torch
import torch.nn as nn


def layernorm_weight_keys(module):
    keys = set()
    for name, m in module.named_modules():
        if isinstance(m, nn.LayerNorm) and m.weight is not None:
            keys.add((name + "." if name else "") + "weight")
    return keys


def fill_params(module, prefix=""):
    """Fill every float parameter of `module` from the recipe (in place).  Returns the list of
    (key, shape) filled, in sorted key order."""
    ln = layernorm_weight_keys(module)
    params = dict(module.named_parameters())
    filled = []
    with torch.no_grad():
        for key in sorted(params):
            p = params[key]
            if key.endswith("logit_scale"):
                filled.append((key, tuple(p.shape)))
                continue
            rng = np.random.default_rng(zlib.crc32((prefix + key).encode()))
            v = rng.standard_normal(tuple(p.shape))
            v = 1.0 + 0.1 * v if key in ln else 0.05 * v
            p.copy_(torch.from_numpy(v.astype(np.float32)))
            filled.append((key, tuple(p.shape)))
    return filled


def randn(seed, shape):
    return np.random.default_rng(seed).standard_normal(shape).astype(np.float32)


def param_signature(module):
    """Sorted (key, shape) of parameters — stored in fixtures to detect drift."""
    return sorted((k, tuple(v.shape)) for k, v in module.named_parameters())
