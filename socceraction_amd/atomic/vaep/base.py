"""Atomic-VAEP on MI355X (drop-in for ``socceraction.atomic.vaep.base``)."""
from typing import Any, List, Optional

from ...vaep.base import VAEP
from .. import spadl as spadlcfg
from . import features as fs
from . import formula as vaep
from . import labels as lab

xfns_default = [
    fs.actiontype,
    fs.actiontype_onehot,
    fs.bodypart,
    fs.bodypart_onehot,
    fs.time,
    fs.team,
    fs.time_delta,
    fs.location,
    fs.polar,
    fs.movement_polar,
    fs.direction,
    fs.goalscore,
]


class AtomicVAEP(VAEP):
    """VAEP for Atomic-SPADL actions (reference atomic/vaep/base.py:34-79)."""

    _spadlcfg = spadlcfg
    _lab = lab
    _fs = fs
    _vaep = vaep
    _atomic = True

    def __init__(self, xfns: Optional[List[Any]] = None, nb_prev_actions: int = 3) -> None:
        xfns = xfns_default if xfns is None else xfns
        super().__init__(xfns, nb_prev_actions)
