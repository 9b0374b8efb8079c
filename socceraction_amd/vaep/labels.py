"""VAEP labels, GPU-backed (drop-in for ``socceraction.vaep.labels``).

The whole input frame is ONE segment, exactly as the reference's shifts ignore
``game_id`` (vaep/labels.py:38-42); use :meth:`VAEP.compute_labels_batch` for many games.
"""
import pandas as pd

from .. import ops
from ..batch import ActionBatch


def _labels(actions: pd.DataFrame, nr_actions: int, atomic: bool):
    if len(actions) == 0:
        return None
    ab = ActionBatch.from_frame(actions, atomic=atomic)
    lb = ops.labels(ab, nr_actions)
    return lb


def _column(actions, nr_actions, atomic, which, name):
    lb = _labels(actions, nr_actions, atomic)
    if lb is None:
        return pd.DataFrame({name: pd.Series([], dtype=bool)}, index=actions.index)
    v = getattr(lb, which)[:len(actions)].cpu().numpy().view(bool)
    return pd.DataFrame({name: v}, index=actions.index)


def scores(actions: pd.DataFrame, nr_actions: int = 10) -> pd.DataFrame:
    """Did the team in possession score within the next ``nr_actions`` actions
    (reference vaep/labels.py:9-50)."""
    return _column(actions, nr_actions, False, 'scores', 'scores')


def concedes(actions: pd.DataFrame, nr_actions: int = 10) -> pd.DataFrame:
    """Did the team in possession concede within the next ``nr_actions`` actions
    (reference vaep/labels.py:53-93)."""
    return _column(actions, nr_actions, False, 'concedes', 'concedes')


def goal_from_shot(actions: pd.DataFrame) -> pd.DataFrame:
    """Was a goal scored from the current action (reference vaep/labels.py:96-116)."""
    return _column(actions, 10, False, 'goal_from_shot', 'goal_from_shot')
