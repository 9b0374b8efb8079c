"""VAEP formula, GPU-backed (drop-in for ``socceraction.vaep.formula``).

The output dtype follows the probability dtype (float32 in -> float32 out), as in the
reference's pandas arithmetic. The whole frame is one segment (``_prev`` ignores
``game_id``, vaep/formula.py:8-11).
"""
import numpy as np
import pandas as pd
import torch

from .. import ops
from ..batch import ActionBatch

_samephase_nb: int = 10


def _probs(x):
    v = x.to_numpy() if isinstance(x, (pd.Series, pd.DataFrame)) else np.asarray(x)
    return v.reshape(-1)


def _value(actions: pd.DataFrame, Pscores, Pconcedes, atomic: bool) -> pd.DataFrame:
    ps, pc = _probs(Pscores), _probs(Pconcedes)
    if len(ps) != len(actions) or len(pc) != len(actions):
        raise ValueError('need one probability per action')
    dt = np.float32 if (ps.dtype == np.float32 and pc.dtype == np.float32) else np.float64
    ps = np.ascontiguousarray(ps, dtype=dt)
    pc = np.ascontiguousarray(pc, dtype=dt)
    n = len(actions)
    cols = ['offensive_value', 'defensive_value', 'vaep_value']
    if n == 0:
        return pd.DataFrame({c: np.zeros(0, dt) for c in cols}, index=actions.index)
    ab = ActionBatch.from_frame(actions, atomic=atomic)
    tps = torch.from_numpy(ps).to(ab.device)
    tpc = torch.from_numpy(pc).to(ab.device)
    out = ops.formula(ab, tps, tpc).cpu().numpy()[:, :n]
    index = Pscores.index if isinstance(Pscores, pd.Series) else actions.index
    return pd.DataFrame({c: out[r] for r, c in enumerate(cols)}, index=index)


def offensive_value(actions: pd.DataFrame, scores, concedes) -> pd.Series:
    """Change in scoring probability (reference vaep/formula.py:17-68)."""
    return _value(actions, scores, concedes, False)['offensive_value'].rename(None)


def defensive_value(actions: pd.DataFrame, scores, concedes) -> pd.Series:
    """Negated change in conceding probability (reference vaep/formula.py:71-113)."""
    return _value(actions, scores, concedes, False)['defensive_value'].rename(None)


def value(actions: pd.DataFrame, Pscores, Pconcedes) -> pd.DataFrame:
    """offensive_value, defensive_value and vaep_value (reference vaep/formula.py:116-151)."""
    return _value(actions, Pscores, Pconcedes, False)
