"""Stand-in for the reference's plugin ABC when this package runs outside the
reference tree.

Inside the viewer the real base class is the reference's ``interface.py``
(``SatellitePlugin``, interface.py:10-47; ``Layer`` tuple type, :5-7) and
``plugin.py`` imports that.  This module restates the same contract so the
plugin can be exercised headless: a ``name`` property, an optional
``requires_viewer`` flag (False by default) and ``run(...) -> list of
(data, params, layer_type)`` tuples where ``layer_type`` is one of
"image" | "labels" | "points" | "shapes".
"""
from __future__ import annotations

from abc import ABC, abstractmethod
from typing import Any, Dict, List, Literal, Tuple

import numpy as np

LayerType = Literal["image", "labels", "points", "shapes"]
LayerParams = Dict[str, Any]
Layer = Tuple[np.ndarray, LayerParams, LayerType]


class SatellitePlugin(ABC):
    @property
    @abstractmethod
    def name(self) -> str:
        """Display name in the viewer."""

    @property
    def requires_viewer(self) -> bool:
        return False

    @abstractmethod
    def run(self, *args, **kwargs) -> List[Layer]:
        """Produce napari layer tuples."""
