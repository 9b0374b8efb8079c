"""SPADL schema (reference ``spadl/schema.py:10-33``, pandera ``SchemaModel``).

pandera is not part of this image, so the schema is a small explicit checker with the
same fields and constraints; :meth:`SPADLSchema.validate` raises ``ValueError`` where
pandera would raise ``SchemaError``.
"""
from typing import Dict, Tuple

import numpy as np
import pandas as pd

from . import config as spadlconfig

# column -> (kind, lo, hi) ; kind 'i' int, 'f' float, 'a' any
FIELDS: Dict[str, Tuple[str, float, float]] = {
    'game_id': ('a', None, None), 'original_event_id': ('a', None, None),
    'action_id': ('i', None, None), 'period_id': ('i', 1, 5), 'time_seconds': ('f', 0, None),
    'team_id': ('a', None, None), 'player_id': ('a', None, None),
    'start_x': ('f', 0, spadlconfig.field_length), 'start_y': ('f', 0, spadlconfig.field_width),
    'end_x': ('f', 0, spadlconfig.field_length), 'end_y': ('f', 0, spadlconfig.field_width),
    'bodypart_id': ('i', 0, len(spadlconfig.bodyparts) - 1),
    'type_id': ('i', 0, len(spadlconfig.actiontypes) - 1),
    'result_id': ('i', 0, len(spadlconfig.results) - 1),
}
OPTIONAL = {'bodypart_name', 'type_name', 'result_name'}


class _Schema:
    fields = FIELDS
    optional = OPTIONAL

    @classmethod
    def cast(cls, df: pd.DataFrame) -> pd.DataFrame:
        """Coerce numeric columns to the schema dtypes (pandera ``coerce=True``)."""
        for c, (kind, _, _) in cls.fields.items():
            if c in df.columns and kind == 'i' and df[c].dtype.kind == 'f' \
                    and not df[c].isna().any():
                df[c] = df[c].astype(np.int64)
            elif c in df.columns and kind == 'f' and df[c].dtype.kind in 'iu':
                df[c] = df[c].astype(np.float64)
        return df

    @classmethod
    def validate(cls, df: pd.DataFrame) -> pd.DataFrame:
        """Check columns and value ranges (pandera ``strict=True`` semantics)."""
        extra = set(df.columns) - set(cls.fields) - cls.optional
        if extra:
            raise ValueError(f'columns not in the schema: {sorted(extra)}')
        for c, (kind, lo, hi) in cls.fields.items():
            if c not in df.columns:
                raise ValueError(f'column {c!r} not in dataframe')
            v = df[c]
            if lo is not None and (v < lo).any():
                raise ValueError(f'{c} has values < {lo}')
            if hi is not None and (v > hi).any():
                raise ValueError(f'{c} has values > {hi}')
        return cls.cast(df)


class SPADLSchema(_Schema):
    """Definition of a SPADL dataframe."""
