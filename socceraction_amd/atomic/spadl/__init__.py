"""Atomic-SPADL vocabulary, schema and helpers (reference ``socceraction/atomic/spadl``).

``convert_to_atomic`` (SPADL -> Atomic-SPADL) is ranked "next" in SURVEY.md §8(f) and is
not part of this round's valuation path.
"""
from . import config
from .config import actiontypes_df, bodyparts_df
from .schema import AtomicSPADLSchema
from .utils import add_names, play_left_to_right

__all__ = ['config', 'AtomicSPADLSchema', 'bodyparts_df', 'actiontypes_df', 'add_names',
           'play_left_to_right']
