"""Atomic-SPADL vocabulary (reference ``atomic/spadl/config.py:19-47``).

The SPADL action types extended with 10 atomic types (ids 23-32). Note that
``'interception'`` appears twice (ids 10 and 24); the reference's one-hot
transformer therefore yields a single ``type_interception`` column that is true
for both ids (reproduced by the kernels' name-id LUT).
"""
import pandas as pd

from ...spadl import config as _spadl

field_length = _spadl.field_length
field_width = _spadl.field_width

bodyparts = _spadl.bodyparts
bodyparts_df = _spadl.bodyparts_df

actiontypes = _spadl.actiontypes + [
    'receival', 'interception', 'out', 'offside', 'goal', 'owngoal', 'yellow_card',
    'red_card', 'corner', 'freekick',
]


def actiontypes_df() -> pd.DataFrame:
    """(type_id, type_name) table for Atomic-SPADL."""
    return pd.DataFrame(list(enumerate(actiontypes)), columns=['type_id', 'type_name'])
