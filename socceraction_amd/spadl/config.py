"""SPADL vocabulary and pitch constants.

Mirrors ``socceraction/spadl/config.py:21-90`` (reference): pitch size, the 23
action types (ids 0-22), 6 results (ids 0-5) and 4 bodyparts (ids 0-3). The
numeric ids are positions in these lists; the HIP kernels hard-code the same ids
in ``csrc/sa_common.h``.
"""
from typing import List

import pandas as pd

field_length: float = 105.0  # metres
field_width: float = 68.0  # metres

bodyparts: List[str] = ['foot', 'head', 'other', 'head/other']
results: List[str] = ['fail', 'success', 'offside', 'owngoal', 'yellow_card', 'red_card']
actiontypes: List[str] = [
    'pass', 'cross', 'throw_in', 'freekick_crossed', 'freekick_short', 'corner_crossed',
    'corner_short', 'take_on', 'foul', 'tackle', 'interception', 'shot', 'shot_penalty',
    'shot_freekick', 'keeper_save', 'keeper_claim', 'keeper_punch', 'keeper_pick_up',
    'clearance', 'bad_touch', 'non_action', 'dribble', 'goalkick',
]


def actiontypes_df() -> pd.DataFrame:
    """(type_id, type_name) table (reference ``spadl/config.py:60-68``)."""
    return pd.DataFrame(list(enumerate(actiontypes)), columns=['type_id', 'type_name'])


def results_df() -> pd.DataFrame:
    """(result_id, result_name) table (reference ``spadl/config.py:71-79``)."""
    return pd.DataFrame(list(enumerate(results)), columns=['result_id', 'result_name'])


def bodyparts_df() -> pd.DataFrame:
    """(bodypart_id, bodypart_name) table (reference ``spadl/config.py:82-90``)."""
    return pd.DataFrame(list(enumerate(bodyparts)), columns=['bodypart_id', 'bodypart_name'])
