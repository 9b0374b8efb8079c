"""Atomic-VAEP formula, GPU-backed (drop-in for ``socceraction.atomic.vaep.formula``).

As the SPADL formula but without the time-gap, penalty and corner rules; the
previous-goal rule tests the previous action's type against goal / owngoal
(atomic/vaep/formula.py:8-141).
"""
import pandas as pd

from ...vaep.formula import _value


def offensive_value(actions: pd.DataFrame, scores, concedes) -> pd.Series:
    """Reference atomic/vaep/formula.py:14-57."""
    return _value(actions, scores, concedes, True)['offensive_value'].rename(None)


def defensive_value(actions: pd.DataFrame, scores, concedes) -> pd.Series:
    """Reference atomic/vaep/formula.py:60-103."""
    return _value(actions, scores, concedes, True)['defensive_value'].rename(None)


def value(actions: pd.DataFrame, Pscores, Pconcedes) -> pd.DataFrame:
    """Reference atomic/vaep/formula.py:106-141."""
    return _value(actions, Pscores, Pconcedes, True)
