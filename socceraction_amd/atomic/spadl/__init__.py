"""Atomic-SPADL vocabulary, schema, helpers and the SPADL -> Atomic-SPADL conversion
(reference ``socceraction/atomic/spadl``). ``convert_to_atomic`` runs on the GPU
(``base.py``)."""
from . import config
from .base import convert_to_atomic
from .config import actiontypes_df, bodyparts_df
from .schema import AtomicSPADLSchema
from .utils import add_names, play_left_to_right

__all__ = ['config', 'convert_to_atomic', 'AtomicSPADLSchema', 'bodyparts_df', 'actiontypes_df', 'add_names',
           'play_left_to_right']
