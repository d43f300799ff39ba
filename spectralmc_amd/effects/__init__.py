"""Path-scheme and normalisation intents of the GBM engine.

The reference defines these in ``src/spectralmc/effects/montecarlo.py:24-35`` next to its
effect-interpreter machinery; only the two enums are part of the hot path's API (the
interpreter is not called by ``train``, ``gbm_trainer.py:1686-1703``).
"""

from __future__ import annotations

from enum import Enum


class PathScheme(str, Enum):
    LOG_EULER = "log_euler"
    SIMPLE_EULER = "simple_euler"


class ForwardNormalization(str, Enum):
    NORMALIZE = "normalize_forwards"
    RAW = "raw_paths"


__all__ = ["PathScheme", "ForwardNormalization"]
