"""`pytest_mock` stand-in over unittest.mock (test infrastructure only)."""
from unittest import mock

import pytest


class MockerFixture:  # noqa: D101
    def __init__(self):
        self._patches = []
        outer = self

        class _Patch:
            def object(self, target, attr, new=mock.DEFAULT, **kw):
                p = mock.patch.object(target, attr, new, **kw)
                outer._patches.append(p)
                return p.start()

        self.patch = _Patch()

    def stopall(self):
        for p in reversed(self._patches):
            p.stop()
        self._patches.clear()


@pytest.fixture
def mocker():
    m = MockerFixture()
    yield m
    m.stopall()
