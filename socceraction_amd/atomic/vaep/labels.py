"""Atomic-VAEP labels, GPU-backed (drop-in for ``socceraction.atomic.vaep.labels``).

goal = type ``goal`` (27), owngoal = type ``owngoal`` (28) — no shot condition
(atomic/vaep/labels.py:27-28); the whole frame is one segment.
"""
import pandas as pd

from ...vaep.labels import _column


def scores(actions: pd.DataFrame, nr_actions: int = 10) -> pd.DataFrame:
    """Reference atomic/vaep/labels.py:9-45."""
    return _column(actions, nr_actions, True, 'scores', 'scores')


def concedes(actions: pd.DataFrame, nr_actions: int = 10) -> pd.DataFrame:
    """Reference atomic/vaep/labels.py:48-84."""
    return _column(actions, nr_actions, True, 'concedes', 'concedes')


def goal_from_shot(actions: pd.DataFrame) -> pd.DataFrame:
    """A shot followed by a goal; False on the last row (atomic/vaep/labels.py:87-107)."""
    return _column(actions, 10, True, 'goal_from_shot', 'goal')
