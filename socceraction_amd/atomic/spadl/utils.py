"""Atomic-SPADL helpers (reference ``atomic/spadl/utils.py``)."""
import pandas as pd

from . import config as spadlconfig
from .schema import AtomicSPADLSchema


def add_names(actions: pd.DataFrame) -> pd.DataFrame:
    """Add type_name and bodypart_name (reference atomic/spadl/utils.py:8-27)."""
    out = (actions.drop(columns=['type_name', 'bodypart_name'], errors='ignore')
           .merge(spadlconfig.actiontypes_df(), how='left')
           .merge(spadlconfig.bodyparts_df(), how='left'))
    return AtomicSPADLSchema.cast(out)


def play_left_to_right(actions: pd.DataFrame, home_team_id) -> pd.DataFrame:
    """Flip away-team atomic actions (reference atomic/spadl/utils.py:30-56)."""
    ltr = actions.copy()
    away = (actions.team_id != home_team_id).to_numpy()
    ltr.loc[away, 'x'] = spadlconfig.field_length - actions.loc[away, 'x'].to_numpy()
    ltr.loc[away, 'y'] = spadlconfig.field_width - actions.loc[away, 'y'].to_numpy()
    ltr.loc[away, 'dx'] = -actions.loc[away, 'dx'].to_numpy()
    ltr.loc[away, 'dy'] = -actions.loc[away, 'dy'].to_numpy()
    return ltr
