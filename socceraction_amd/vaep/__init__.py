"""VAEP (drop-in for ``socceraction.vaep``)."""
from . import features, formula, labels
from .base import VAEP

__all__ = ['VAEP', 'features', 'labels', 'formula']
