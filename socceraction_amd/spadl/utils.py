"""SPADL DataFrame helpers (reference ``spadl/utils.py``).

These are host-side DataFrame plumbing (string-name joins and row copies), not
valuation arithmetic; the valuation kernels work on ids and never need them.
"""
import pandas as pd

from . import config as spadlconfig
from .schema import SPADLSchema


def add_names(actions: pd.DataFrame) -> pd.DataFrame:
    """Add type_name, result_name and bodypart_name (reference spadl/utils.py:8-28).

    Left-joins the vocabulary tables; the result has a fresh RangeIndex like the
    reference's ``merge``.
    """
    out = (actions.drop(columns=['type_name', 'result_name', 'bodypart_name'], errors='ignore')
           .merge(spadlconfig.actiontypes_df(), how='left')
           .merge(spadlconfig.results_df(), how='left')
           .merge(spadlconfig.bodyparts_df(), how='left'))
    return SPADLSchema.cast(out)


def play_left_to_right(actions: pd.DataFrame, home_team_id=None) -> pd.DataFrame:
    """Flip away-team actions so every team plays left to right.

    Mirrors reference spadl/utils.py:59-80 (which reads a ``home_team_id`` column);
    the two-argument form of spadl/utils.py:31-57 is accepted too.
    """
    ltr = actions.copy()
    home = actions['home_team_id'] if home_team_id is None else home_team_id
    away = (actions.team_id != home).to_numpy()
    for col in ('start_x', 'end_x'):
        ltr.loc[away, col] = spadlconfig.field_length - actions.loc[away, col].to_numpy()
    for col in ('start_y', 'end_y'):
        ltr.loc[away, col] = spadlconfig.field_width - actions.loc[away, col].to_numpy()
    return ltr


def play_left_to_right_sa(actions: pd.DataFrame, home_team_id: int) -> pd.DataFrame:
    """Two-argument form of reference spadl/utils.py:31-57 (away-team rows flipped)."""
    return play_left_to_right(actions, home_team_id)
