"""Atomic-VAEP (drop-in for ``socceraction.atomic.vaep``)."""
from . import features, formula, labels
from .base import AtomicVAEP

__all__ = ['AtomicVAEP', 'features', 'labels', 'formula']
