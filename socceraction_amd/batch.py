"""Columnar action batches in HBM: the boundary between pandas and the HIP kernels.

A SPADL / Atomic-SPADL DataFrame is flattened ONCE into device columns:

=============  =======  ===============================================================
column         dtype    notes
=============  =======  ===============================================================
c0..c3         float64  SPADL start_x, start_y, end_x, end_y / atomic x, y, dx, dy
time_seconds   float64
type_id        uint8    SPADL 0-22, atomic 0-32 (validated like SPADLSchema's isin)
result_id      uint8    SPADL only, 0-5
bodypart_id    uint8    0-3
period_id      uint8    1-5
team           int32    factorised team ids (equality-preserving codes)
seg_off        int64    [n_segments + 1] segment (game) offsets
home_team      int32    [n_segments] code of each segment's home team (or absent)
=============  =======  ===============================================================

All columns of one batch live in ONE device allocation carved at 256-byte aligned
offsets (one host->device copy per batch). :func:`ActionBatch.struct` produces the
``sa_actions`` C struct of ``include/socceraction_amd.h``.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence

import numpy as np
import pandas as pd
import torch

from ._native import SA_MAX_FRAMES, SaActions
from .atomic.spadl import config as atomicconfig
from .spadl import config as spadlconfig

_ALIGN = 256
F64_COLS_SPADL = ('start_x', 'start_y', 'end_x', 'end_y')
F64_COLS_ATOMIC = ('x', 'y', 'dx', 'dy')


def device() -> torch.device:
    """The current ROCm device; raises when there is none (no CPU fallback)."""
    if not torch.cuda.is_available():
        raise RuntimeError('socceraction_amd requires a ROCm GPU (MI355X / gfx950); '
                           'none is visible to torch.')
    return torch.device('cuda', torch.cuda.current_device())


def stream_handle() -> int:
    return torch.cuda.current_stream().cuda_stream


def _round(n: int, a: int) -> int:
    return (n + a - 1) // a * a


def _ids(df: pd.DataFrame, col: str, names: Optional[List[str]], lo: int, hi: int,
         required: bool = True) -> np.ndarray:
    n = len(df)
    if col in df.columns:
        v = df[col].to_numpy()
    elif names is not None and col.replace('_id', '_name') in df.columns:
        lut = {name: i for i, name in enumerate(names)}
        v = df[col.replace('_id', '_name')].map(lut).to_numpy()
    elif not required:
        return np.full(n, lo, dtype=np.uint8)
    else:
        raise ValueError(f'column {col} is missing from the actions dataframe')
    if v.dtype.kind == 'f':
        if np.isnan(v).any():
            raise ValueError(f'{col} contains NaN')
        if (v != np.floor(v)).any():
            raise ValueError(f'{col} must hold integers')
    elif v.dtype.kind not in 'iub':
        v = pd.to_numeric(pd.Series(v), errors='raise').to_numpy()
    if n and (v.min() < lo or v.max() > hi):
        raise ValueError(f'{col} values must lie in [{lo}, {hi}] (SPADL schema isin check)')
    return v.astype(np.uint8)


def _f64(df: pd.DataFrame, col: str, required: bool = True) -> np.ndarray:
    if col not in df.columns:
        if required:
            raise ValueError(f'column {col} is missing from the actions dataframe')
        return np.zeros(len(df))
    return np.ascontiguousarray(df[col].to_numpy(dtype=np.float64))


def encode_teams(team_ids: np.ndarray, home_ids: Sequence = ()) -> tuple:
    """Equality-preserving int32 codes for team ids (and for the home-team ids)."""
    team_ids = np.asarray(team_ids)
    home_ids = np.asarray(list(home_ids))
    if team_ids.dtype.kind in 'iu' and (home_ids.size == 0 or home_ids.dtype.kind in 'iu'):
        lo = min(team_ids.min(initial=0), home_ids.min(initial=0))
        hi = max(team_ids.max(initial=0), home_ids.max(initial=0))
        if lo >= -2**31 and hi < 2**31:
            return team_ids.astype(np.int32), home_ids.astype(np.int32)
    codes, uniques = pd.factorize(pd.Series(team_ids), use_na_sentinel=True)
    if (codes < 0).any():
        raise ValueError('team_id contains missing values')
    index = pd.Index(uniques)
    hc = np.array([index.get_loc(h) if h in index else -1 for h in home_ids], dtype=np.int32)
    return codes.astype(np.int32), hc


def segment_offsets(game_id: np.ndarray) -> np.ndarray:
    """Offsets of the contiguous runs of equal ``game_id`` values."""
    n = len(game_id)
    if n == 0:
        return np.zeros(1, dtype=np.int64)
    change = np.flatnonzero(np.asarray(game_id[1:]) != np.asarray(game_id[:-1])) + 1
    return np.concatenate([[0], change, [n]]).astype(np.int64)


class ActionBatch:
    """Device-resident columns of one frame of actions (see module docstring)."""

    def __init__(self, cols: Dict[str, np.ndarray], seg_off: np.ndarray,
                 home: Optional[np.ndarray], atomic: bool, dev: Optional[torch.device] = None,
                 contiguous: bool = False, pinned: bool = False):
        dev = dev or device()
        self.atomic = bool(atomic)
        self.n = int(len(cols['type_id']))
        self.n_segments = int(len(seg_off) - 1)
        if seg_off[0] != 0 or seg_off[-1] != self.n or (np.diff(seg_off) < 0).any():
            raise ValueError('segment offsets must start at 0, end at n and be non-decreasing')
        order = ['c0', 'c1', 'c2', 'c3', 'time_seconds', 'team', 'type_id', 'result_id',
                 'bodypart_id', 'period_id']
        arrays = {k: np.ascontiguousarray(cols[k]) for k in order if k in cols}
        arrays['seg_off'] = np.ascontiguousarray(seg_off, dtype=np.int64)
        if home is not None:
            arrays['home'] = np.ascontiguousarray(home, dtype=np.int32)
        offsets, total = {}, 0
        for k, a in arrays.items():
            offsets[k] = total
            total += _round(max(a.nbytes, 16), _ALIGN)
        # pinned: the host image in page-locked memory and the H2D asynchronous on the current
        # stream (the image is kept with the batch) -- a pageable H2D is staged by the runtime
        # and waits for the DMA engine behind any device-to-host copy in flight
        # (socceraction_amd.pipeline overlaps its D2H with the next chunk's H2D)
        hostt = torch.zeros(total, dtype=torch.uint8, pin_memory=True) if pinned else None
        host = hostt.numpy() if pinned else np.zeros(total, dtype=np.uint8)
        for k, a in arrays.items():
            host[offsets[k]:offsets[k] + a.nbytes] = a.view(np.uint8).reshape(-1)
        self._dbuf = None
        self._host = hostt
        if contiguous:  # one physically contiguous range (``ops.DeviceBuffer``), raises if none
            from .ops import DeviceBuffer
            self._dbuf = DeviceBuffer(total, contiguous=True)
            self.buffer = self._dbuf.tensor((total,), torch.uint8)
            self.buffer.copy_(torch.from_numpy(host))
        elif pinned:
            self.buffer = torch.empty(total, dtype=torch.uint8, device=dev)
            self.buffer.copy_(hostt, non_blocking=True)
        else:
            self.buffer = torch.from_numpy(host).to(dev)
        self.cols: Dict[str, torch.Tensor] = {}
        for k, a in arrays.items():
            o = offsets[k]
            self.cols[k] = self.buffer[o:o + a.nbytes].view(torch.from_numpy(a[:0]).dtype) \
                if a.nbytes else torch.empty(0, dtype=torch.from_numpy(a[:0]).dtype, device=dev)
        self.device = dev
        self._seg_blocks()  # now, on the stream that copied seg_off: struct() never launches

    # ------------------------------------------------------------------ constructors
    @classmethod
    def from_frame(cls, df: pd.DataFrame, *, atomic: bool = False, home_team_id=None,
                   segments: str = 'single', team_codes=None, dev=None,
                   pinned: bool = False) -> 'ActionBatch':
        """Flatten a SPADL / Atomic-SPADL frame.

        ``segments='single'``: the whole frame is one segment (the reference's
        module-level semantics). ``segments='game'``: one segment per contiguous run
        of ``game_id``; ``home_team_id`` is then a per-segment sequence (or a mapping
        ``game_id -> home_team_id``).
        """
        cols = encode_columns(df, atomic)
        n = len(df)
        if segments == 'single':
            seg_off = np.array([0, n], dtype=np.int64)
            homes = [] if home_team_id is None else [home_team_id]
        elif segments == 'game':
            seg_off = segment_offsets(df['game_id'].to_numpy())
            if home_team_id is None:
                homes = []
            elif isinstance(home_team_id, pd.Series):  # one vectorised lookup (KeyError if absent)
                gids = df['game_id'].to_numpy()[seg_off[:-1]]
                homes = list(home_team_id.loc[gids]) if len(gids) else []
            elif isinstance(home_team_id, dict):
                gids = df['game_id'].to_numpy()[seg_off[:-1]]
                homes = [home_team_id[g] for g in gids]
            else:
                homes = list(home_team_id)
                if len(homes) != len(seg_off) - 1:
                    raise ValueError('need one home_team_id per game segment')
        else:
            raise ValueError("segments must be 'single' or 'game'")
        if team_codes is not None:
            cols['team'], hc = team_codes
        else:
            cols['team'], hc = encode_teams(df['team_id'].to_numpy(), homes)
        home = hc if homes else None
        return cls(cols, seg_off, home, atomic, dev, pinned=pinned)

    @classmethod
    def from_columns(cls, d: Dict[str, np.ndarray], *, atomic: bool = False,
                     flip: bool = True, dev=None, contiguous: bool = False) -> 'ActionBatch':
        """From the flat numpy columns of :mod:`socceraction_amd.synthetic` (``contiguous``:
        the device buffer in physically contiguous VRAM, see ``ActionBatch.__init__``)."""
        f64 = F64_COLS_ATOMIC if atomic else F64_COLS_SPADL
        cols = {f'c{i}': np.asarray(d[c], dtype=np.float64) for i, c in enumerate(f64)}
        cols['time_seconds'] = np.asarray(d['time_seconds'], dtype=np.float64)
        cols['type_id'] = np.asarray(d['type_id'], dtype=np.uint8)
        if not atomic:
            cols['result_id'] = np.asarray(d['result_id'], dtype=np.uint8)
        cols['bodypart_id'] = np.asarray(d['bodypart_id'], dtype=np.uint8)
        cols['period_id'] = np.asarray(d['period_id'], dtype=np.uint8)
        team, home = encode_teams(d['team_id'], d['home_team_id'])
        cols['team'] = team
        return cls(cols, np.asarray(d['game_off'], dtype=np.int64), home if flip else None,
                   atomic, dev, contiguous)

    @classmethod
    def from_device(cls, cols: Dict[str, torch.Tensor], n: int, seg_off: torch.Tensor,
                    home: Optional[torch.Tensor], atomic: bool) -> 'ActionBatch':
        """Wrap columns already in HBM (16-byte aligned; kernel dtypes of the module table),
        e.g. the output of the device SPADL -> Atomic-SPADL conversion. No copy."""
        self = cls.__new__(cls)
        self.atomic = bool(atomic)
        self.n = int(n)
        self.n_segments = int(seg_off.numel() - 1)
        self.cols = dict(cols)
        self.cols['seg_off'] = seg_off
        if home is not None:
            self.cols['home'] = home
        self.buffer = None
        self.device = seg_off.device
        self._seg_blocks()  # now, on the stream that wrote seg_off (the caller's current one)
        return self

    # ------------------------------------------------------------------ C structs
    def _frame(self, fr) -> None:
        c = self.cols
        ptr = lambda k: c[k].data_ptr() if k in c else None  # noqa: E731
        fr.c0, fr.c1, fr.c2, fr.c3 = ptr('c0'), ptr('c1'), ptr('c2'), ptr('c3')
        fr.time_seconds = ptr('time_seconds')
        fr.type_id, fr.result_id = ptr('type_id'), ptr('result_id')
        fr.bodypart_id, fr.period_id, fr.team = ptr('bodypart_id'), ptr('period_id'), ptr('team')

    def _seg_blocks(self) -> Optional[int]:
        """Device pointer of the segment of every SA_SEG_BLOCK-row block (``sa_segment_blocks``),
        or None for a single segment (nothing to search).  Built once, when the batch is made, on
        the stream current then (the one that wrote seg_off), and host-synchronised there, so any
        stream may read it and struct() -- called inside timed regions and under other streams --
        never launches or synchronises."""
        if self.n_segments <= 1 or self.n == 0:
            return None
        t = self.cols.get('seg_of_block')
        if t is None:
            from . import _native
            t = torch.empty(-(-self.n // _native.SA_SEG_BLOCK), dtype=torch.int32, device=self.device)
            st = torch.cuda.current_stream()
            _native.check(_native.lib().sa_segment_blocks(self.cols['seg_off'].data_ptr(), self.n_segments,
                                                          self.n, t.data_ptr(), st.cuda_stream))
            st.synchronize()  # once per batch: every stream may use the table afterwards
            self.cols['seg_of_block'] = t
        return t.data_ptr()

    def struct(self, flip: bool = True) -> SaActions:
        s = SaActions()
        s.n = self.n
        s.n_segments = self.n_segments
        s.seg_off = self.cols['seg_off'].data_ptr()
        s.seg_of_block = self._seg_blocks()
        s.home_team = self.cols['home'].data_ptr() if (flip and 'home' in self.cols) else None
        s.n_frames = 1
        s.atomic = int(self.atomic)
        self._frame(s.frames[0])
        return s

    @staticmethod
    def explicit_struct(frames: Sequence['ActionBatch']) -> SaActions:
        """Explicit-frame mode: window i of row j = row j of frames[i] (one segment)."""
        if not 1 <= len(frames) <= SA_MAX_FRAMES:
            raise ValueError(f'between 1 and {SA_MAX_FRAMES} game-state frames are supported')
        n = frames[0].n
        if any(f.n != n for f in frames):
            raise ValueError('all game-state frames must have the same length')
        s = frames[0].struct(flip=False)
        s.n_frames = len(frames)
        for i, f in enumerate(frames):
            f._frame(s.frames[i])
        return s


def encode_columns(df: pd.DataFrame, atomic: bool) -> Dict[str, np.ndarray]:
    """Validate + convert the numeric input columns of one frame to kernel dtypes."""
    f64 = F64_COLS_ATOMIC if atomic else F64_COLS_SPADL
    cols = {f'c{i}': _f64(df, c, required=False) for i, c in enumerate(f64)}
    cols['time_seconds'] = _f64(df, 'time_seconds', required=False)
    if atomic:
        cols['type_id'] = _ids(df, 'type_id', atomicconfig.actiontypes, 0,
                               len(atomicconfig.actiontypes) - 1)
    else:
        cols['type_id'] = _ids(df, 'type_id', spadlconfig.actiontypes, 0,
                               len(spadlconfig.actiontypes) - 1)
        cols['result_id'] = _ids(df, 'result_id', spadlconfig.results, 0,
                                 len(spadlconfig.results) - 1, required=False)
    cols['bodypart_id'] = _ids(df, 'bodypart_id', spadlconfig.bodyparts, 0, 3, required=False)
    cols['period_id'] = _ids(df, 'period_id', None, 1, 5, required=False)
    return cols


def frames_batches(frames: Sequence[pd.DataFrame], atomic: bool, dev=None) -> List[ActionBatch]:
    """One batch per game-state frame, with team codes factorised jointly."""
    team_all = np.concatenate([f['team_id'].to_numpy() if 'team_id' in f.columns
                               else np.zeros(len(f), np.int64) for f in frames])
    codes, _ = encode_teams(team_all)
    out, o = [], 0
    for f in frames:
        n = len(f)
        out.append(ActionBatch.from_frame(
            f, atomic=atomic, team_codes=(codes[o:o + n], np.zeros(0, np.int32)), dev=dev))
        o += n
    return out
