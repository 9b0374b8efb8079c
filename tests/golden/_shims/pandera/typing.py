"""`pandera.typing` stand-in: generic aliases resolve to plain pandas classes."""
import pandas as pd


class DataFrame(pd.DataFrame):  # noqa: D101
    def __class_getitem__(cls, item):
        return pd.DataFrame


class Series(pd.Series):  # noqa: D101
    def __class_getitem__(cls, item):
        return pd.Series


class Index(pd.Index):  # noqa: D101
    def __class_getitem__(cls, item):
        return pd.Index
