"""Atomic-SPADL schema (reference ``atomic/spadl/schema.py:10-31``)."""
from ...spadl.schema import _Schema
from . import config as spadlconfig

FIELDS = {
    'game_id': ('a', None, None), 'original_event_id': ('a', None, None),
    'action_id': ('i', None, None), 'period_id': ('i', 1, 5), 'time_seconds': ('f', 0, None),
    'team_id': ('a', None, None), 'player_id': ('a', None, None),
    'x': ('f', 0, spadlconfig.field_length), 'y': ('f', 0, spadlconfig.field_width),
    'dx': ('f', -spadlconfig.field_length, spadlconfig.field_length),
    'dy': ('f', -spadlconfig.field_width, spadlconfig.field_width),
    'bodypart_id': ('i', 0, len(spadlconfig.bodyparts) - 1),
    'type_id': ('i', 0, len(spadlconfig.actiontypes) - 1),
}


class AtomicSPADLSchema(_Schema):
    """Definition of an Atomic-SPADL dataframe."""

    fields = FIELDS
    optional = {'bodypart_name', 'type_name'}
