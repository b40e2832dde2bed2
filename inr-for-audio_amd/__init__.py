"""MI355X-native SIREN audio fitting (the senyuanfan/inr-for-audio hot path).

Public API mirrors the reference: ``models.SineLayer`` / ``models.SirenWithSnakeTanh``
(models.py), ``run.train`` (run.py) and ``utils`` (get_coord, WaveformFitting,
calculate_snr).  Compute goes through libsiren_hip.so (hand-written gfx950 HIP kernels).
"""
from . import _lib, engine, models, run, utils  # noqa: F401
from .engine import SirenEngine  # noqa: F401
from .models import SineLayer, SirenWithSnakeTanh  # noqa: F401
from .run import train  # noqa: F401

__all__ = ["SineLayer", "SirenWithSnakeTanh", "SirenEngine", "train", "models", "run", "utils",
           "engine"]
