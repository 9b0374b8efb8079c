"""SPADL vocabulary, schema and helpers (reference ``socceraction/spadl``).

Only the parts the valuation path needs; the provider converters (StatsBomb, Opta,
Wyscout) are out of scope.
"""
from . import config
from .config import actiontypes_df, bodyparts_df, results_df
from .schema import SPADLSchema
from .utils import add_names, play_left_to_right

__all__ = ['config', 'SPADLSchema', 'bodyparts_df', 'actiontypes_df', 'results_df', 'add_names',
           'play_left_to_right']
