"""Minimal local stand-in for `pandera` (not installed in this image).

Test infrastructure only: used by tests/golden/make_golden.py to import the
read-only reference for golden-vector generation. `DataFrame[Schema]` is a
no-op cast; the generator asserts schema conditions (dtypes, ranges) itself.
"""
from typing import Any


class SchemaModel:  # noqa: D101
    pass


DataFrameModel = SchemaModel


def Field(*args: Any, **kwargs: Any) -> None:  # noqa: N802,D103
    return None


def check(*args: Any, **kwargs: Any):  # noqa: D103
    def deco(fn):
        return fn
    return deco


dataframe_check = check

from . import typing  # noqa: E402,F401
