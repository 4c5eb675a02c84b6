"""Platform-independent parameter recipe shared by the golden generator, the oracle and the tests.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py): nothing on the product path imports this.

Every state-dict entry is drawn from its own numpy PCG64 stream seeded with
``[seed, crc32(key)]`` (SURVEY.md §8c "Fixtures to generate"), so a fixture stores only the seed
and the recipe, never the 69 MB of weights, and the same tensors come out on any host.

* 5-D conv weight  ``[Cout, Cin/groups, k, k, k]``  ->  N(0,1) / sqrt(Cin/groups * k^3)
* 1-D ``*.weight`` (GroupNorm gamma)               ->  1 + 0.1 N(0,1)
* 1-D ``*.bias``   (GroupNorm beta, conv bias)     ->  0.1 N(0,1)
* 2-D Linear weight ``[out, in]``                   ->  N(0,1) / sqrt(in)
* class tokens (plain tensors, not state_dict)      ->  N(0,1)   (``torch.randn``, unet3D.py:1016-1021)
"""
import zlib

import numpy as np


def param_array(key: str, shape, seed: int = 0) -> np.ndarray:
    rng = np.random.default_rng([seed, zlib.crc32(key.encode())])
    shape = tuple(int(s) for s in shape)
    z = rng.standard_normal(shape)
    if len(shape) == 5:
        fan_in = shape[1] * shape[2] * shape[3] * shape[4]
        out = z / np.sqrt(fan_in)
    elif len(shape) == 2 and key.startswith("class_token"):
        out = z
    elif len(shape) == 2:
        out = z / np.sqrt(shape[1])
    elif len(shape) == 1 and key.endswith("weight"):
        out = 1.0 + 0.1 * z
    elif len(shape) == 1 and key.endswith("bias"):
        out = 0.1 * z
    else:
        raise ValueError(f"weights_recipe: no rule for {key} {shape}")
    return out.astype(np.float32)


def recipe_state_dict(shapes, seed: int = 0):
    """``shapes``: ordered iterable of (key, shape). Returns {key: np.float32 array}."""
    return {k: param_array(k, s, seed) for k, s in shapes}


def apply_recipe(module, seed: int = 0):
    """Overwrite every parameter of a torch module in place with the recipe values."""
    import torch

    sd = module.state_dict()
    new = {k: torch.from_numpy(param_array(k, v.shape, seed)) for k, v in sd.items()}
    module.load_state_dict(new)
    return module


def input_volume(shape, seed: int = 0, kind: str = "normal") -> np.ndarray:
    """Seeded synthetic input volume (fp32). ``kind``: 'normal' = N(0,1) (MRI z-scored),
    'ct' = U(-1000, 1000) HU clipped to +-325 then /325 (MOTSDataset.py:171-182)."""
    rng = np.random.default_rng([seed, 0xC0FFEE])
    if kind == "normal":
        return rng.standard_normal(shape).astype(np.float32)
    if kind == "ct":
        hu = rng.uniform(-1000.0, 1000.0, size=shape)
        return (np.clip(hu, -325.0, 325.0) / 325.0).astype(np.float32)
    raise ValueError(kind)


def label_volume(shape, n_classes: int, seed: int = 0) -> np.ndarray:
    rng = np.random.default_rng([seed, 0x1ABE1])
    return rng.integers(0, n_classes, size=shape).astype(np.float32)
