"""u3d — MI355X-native (gfx950) executor for the multimodal-PL 3D U-Net path.

The public, drop-in API is the reference's own module layout one level up (unet3D.py, engine.py,
loss_functions/, evaluate_amos.py, utils.py). This package holds the ctypes binding of libu3d.so
(_lib), tensor wrappers (ops), the trunk executor (trunk) and the sub-module runner (subgraph).
"""
from ._lib import LIB_PATH, U3DError, lib  # noqa: F401
