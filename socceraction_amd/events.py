"""Device events without the system-scope fence (``sa_event_*``, csrc/sa_api.hip).

A default HIP event (and every ``torch.cuda.Event``) performs a system-scope release when it
is recorded: the GPU's caches are written back and invalidated so that the host or a peer
device could read what the stream produced.  Between two streams of the SAME device that is
not needed -- every kernel boundary already releases to the device -- and on MI355X it costs
several microseconds per record plus the refill of the caches the next kernel finds cold.
These events are created with ``hipEventDisableSystemFence``; the API mirrors
``torch.cuda.Event`` (record / wait / elapsed_time / synchronize) so the bench step can use
either kind.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch

from . import _native


def _handle(stream: Optional[torch.cuda.Stream]) -> int:
    return (stream if stream is not None else torch.cuda.current_stream()).cuda_stream


class DeviceEvent:
    """A device-local stream-ordering (``enable_timing=False``) or timing event."""

    __slots__ = ('_ev', '_lib')

    def __init__(self, enable_timing: bool = False):
        self._lib = _native.lib()
        ev = ctypes.c_void_p()
        _native.check(self._lib.sa_event_create(1 if enable_timing else 0, ctypes.byref(ev)))
        self._ev = ev

    def record(self, stream: Optional[torch.cuda.Stream] = None) -> 'DeviceEvent':
        _native.check(self._lib.sa_event_record(self._ev, _handle(stream)))
        return self

    def wait(self, stream: Optional[torch.cuda.Stream] = None) -> None:
        """Make ``stream`` (default: the current stream) wait for this event."""
        _native.check(self._lib.sa_stream_wait_event(_handle(stream), self._ev))

    def synchronize(self) -> None:
        _native.check(self._lib.sa_event_synchronize(self._ev))

    def elapsed_time(self, end: 'DeviceEvent') -> float:
        ms = ctypes.c_float()
        _native.check(self._lib.sa_event_elapsed(self._ev, end._ev, ctypes.byref(ms)))
        return float(ms.value)

    def __del__(self):
        ev, lib = getattr(self, '_ev', None), getattr(self, '_lib', None)
        if ev is not None and ev.value and lib is not None:
            lib.sa_event_destroy(ev)
