"""Device-level operations: allocate HBM outputs and launch the C-ABI kernels.

Everything here works on :class:`~socceraction_amd.batch.ActionBatch` objects and
returns torch tensors that stay on the GPU; the pandas-facing drop-in modules
(``vaep``, ``atomic.vaep``, ``xthreat``) are thin wrappers around these calls.
Kernels run on torch's current stream.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _native
from .batch import ActionBatch, stream_handle
from .catalog import FeaturePlan, assemble_frame, build_plan


def _ld(n: int) -> int:
    return max(16, (n + 15) // 16 * 16)


@dataclass
class FeatureBlocks:
    """Feature blocks in HBM, one per dtype, in the tiled column-major layout of
    ``include/socceraction_amd.h``: tensors ``[n_tiles, n_cols, R]`` (R = rows per tile; a
    single tile of R >= n rows is plain column-major). ``Rb`` is the bool block's tile,
    ``Rn`` the f64 / i64 blocks' tile."""

    plan: FeaturePlan
    n: int
    Rb: int
    Rn: int
    bool_block: Optional[torch.Tensor]
    f64_block: torch.Tensor
    i64_block: torch.Tensor
    # bitmap form (features(..., bool_bits=True), the on-device VAEP.rate): the bool features
    # as Arrow bitmaps [n_bool, words] int64 (bit i of word w = row 64w + i) instead of a block
    bool_bits: Optional[torch.Tensor] = None

    @property
    def num32(self) -> bool:
        """True when the f64 / i64 blocks hold float32 values (features(..., num32=True): the
        on-device VAEP.rate of xgboost learners, which compare float32 values)."""
        return self.f64_block.dtype == torch.float32

    @property
    def device(self):
        return self.f64_block.device

    def _blk(self, kind: str) -> torch.Tensor:
        if kind == 'b' and self.bool_block is None:
            self.bool_block = self._unpacked_bools()
            self.Rb = self.bool_block.shape[2]
        return {'b': self.bool_block, 'f': self.f64_block, 'i': self.i64_block}[kind]

    def _unpacked_bools(self) -> torch.Tensor:
        """A one-tile bool block [1, n_bool, ld] of the bitmaps (for host export)."""
        ld = _ld(self.n)
        bits = self.bool_bits.view(torch.uint8)[:, :ld // 8]
        shifts = torch.arange(8, device=bits.device, dtype=torch.uint8)
        out = ((bits.unsqueeze(-1) >> shifts) & 1).reshape(bits.shape[0], -1)[:, :ld]
        return out.unsqueeze(0).contiguous()

    def block(self, kind: str) -> torch.Tensor:
        """``[n_cols, n]`` view (one tile) or untiled copy (several tiles), on device."""
        t = self._blk(kind)
        if t.shape[0] == 1:
            return t[0, :, :self.n]
        return t.permute(1, 0, 2).reshape(t.shape[1], -1)[:, :self.n]

    def column(self, kind: str, col: int) -> torch.Tensor:
        return self._blk(kind)[:, col, :].reshape(-1)[:self.n]

    def rows(self, kind: str, start: int, stop: int) -> torch.Tensor:
        """``[n_cols, stop - start]`` copy of a row range (one game), on device: only the tiles
        that hold those rows are untiled."""
        t = self._blk(kind)
        R = t.shape[2]
        t0, t1 = start // R, max(start, stop - 1) // R + 1
        sub = t[t0:t1].permute(1, 0, 2).reshape(t.shape[1], -1)
        return sub[:, start - t0 * R:stop - t0 * R]

    def to_numpy(self):
        """Host copies ``[n_cols, >= n]`` of the three blocks: whole tiles are copied (one
        contiguous D2H per block into pinned memory, all three in flight together) and the
        padding rows are sliced off on the host."""
        hosts = []
        for k in 'bfi':
            t = self._blk(k)
            src = t[0] if t.shape[0] == 1 else t.permute(1, 0, 2).reshape(t.shape[1], -1)
            h = torch.empty(src.shape, dtype=src.dtype, pin_memory=True)
            h.copy_(src, non_blocking=True)
            hosts.append(h)
        torch.cuda.current_stream().synchronize()
        return tuple(h.numpy()[:, :self.n] for h in hosts)

    def to_frame(self, index=None):
        """Copy to host and build the reference-shaped DataFrame."""
        b, f, i = self.to_numpy()
        return assemble_frame(self.plan, b, f, i, self.n, index)

    def sa_blocks(self):
        """The three ``sa_block`` descriptors of the C ABI."""
        out = []
        if self.bool_block is None:  # bitmap form: the bool descriptor only carries the count
            b = _native.SaBlock()
            b.data, b.n_cols, b.tile_rows = None, self.plan.n_bool, 1024
            out.append(b)
        for t, R in (((self.bool_block, self.Rb),) if self.bool_block is not None else ()) + (
                (self.f64_block, self.Rn), (self.i64_block, self.Rn)):
            # the kernels write ceil(n / R) whole [C, R] tiles: the tensor must hold them
            if (t.dim() != 3 or t.shape[2] != R or t.shape[0] * R < self.n
                    or not t.is_contiguous()):
                raise ValueError(f'feature block of shape {tuple(t.shape)} cannot hold {self.n} '
                                 f'rows in tiles of {R}')
            b = _native.SaBlock()
            b.data = _ptr(t)
            b.n_cols = t.shape[1]
            b.tile_rows = R
            out.append(b)
        return out


def alloc_feature_blocks(plan: FeaturePlan, n: int, dev, bool_tile: Optional[int] = None,
                         num_tile: Optional[int] = None, contiguous: bool = False) -> FeatureBlocks:
    """Allocate the three blocks; a ``None`` tile = one tile (plain column-major).
    ``contiguous``: the bool block in physically contiguous VRAM (``sa_device_alloc``, the
    largest translation fragments: a bool pass that follows another kernel refills fewer
    translations, 1.40 vs 1.50 ms at cfg2 on the boxes measured) -- for long-lived blocks (a
    batch pipeline); falls back to the caching allocator when no contiguous range is free
    (``contiguous='require'``: raises instead).  ``FeatureBlocks.bool_alloc`` says which
    allocator served the bool block: 'contiguous' or 'caching'."""
    Rb = _ld(n) if bool_tile is None else int(bool_tile)
    Rn = _ld(n) if num_tile is None else int(num_tile)
    tb, tn = max(1, -(-n // Rb)), max(1, -(-n // Rn))
    bshape = (tb, plan.n_bool, Rb)
    if contiguous == 'all':  # A/B knob: the three blocks in ONE physically contiguous range
        fshape, ishape = (tn, plan.n_f64, Rn), (tn, plan.n_i64, Rn)
        al = lambda b: -(-b // (2 << 20)) * (2 << 20)  # noqa: E731  (2 MiB aligned parts)
        sizes = [int(np.prod(bshape)), 8 * int(np.prod(fshape)), 8 * int(np.prod(ishape))]
        try:
            arena = DeviceBuffer(al(sizes[0]) + al(sizes[1]) + max(sizes[2], 16), contiguous=True)
        except (RuntimeError, ValueError, _native.NativeError):
            arena = None
        if arena is not None:
            out = FeatureBlocks(plan, n, Rb, Rn, arena.tensor(bshape, torch.uint8),
                                arena.tensor(fshape, torch.float64, al(sizes[0])),
                                arena.tensor(ishape, torch.int64, al(sizes[0]) + al(sizes[1])))
            out._arena = arena
            out.bool_alloc = 'contiguous-all'
            return out
    arena = None
    if contiguous and plan.n_bool:
        try:
            arena = DeviceBuffer(int(np.prod(bshape)), contiguous=True)
        except (RuntimeError, ValueError, _native.NativeError, MemoryError):
            if contiguous == 'require':
                raise
            arena = None
    bblk = arena.tensor(bshape, torch.uint8) if arena is not None else \
        torch.empty(bshape, dtype=torch.uint8, device=dev)
    out = FeatureBlocks(plan, n, Rb, Rn, bblk,
                        torch.empty((tn, plan.n_f64, Rn), dtype=torch.float64, device=dev),
                        torch.empty((tn, plan.n_i64, Rn), dtype=torch.int64, device=dev))
    out._arena = arena  # keeps the contiguous allocation alive with the blocks
    out.bool_alloc = 'contiguous' if arena is not None else 'caching'
    return out


class DeviceBuffer:
    """Device memory from ``sa_device_alloc`` (``contiguous``: physically contiguous VRAM), freed
    when the object goes away; ``tensor(shape, dtype)`` views it through
    ``__cuda_array_interface__`` (no copy)."""

    _typestr = {torch.uint8: '|u1', torch.int32: '<i4', torch.int64: '<i8', torch.float32: '<f4',
                torch.float64: '<f8'}

    def __init__(self, nbytes: int, contiguous: bool = True):
        p = ctypes.c_void_p()
        _native.check(_native.lib().sa_device_alloc(int(nbytes), 1 if contiguous else 0, ctypes.byref(p)))
        self.ptr, self.nbytes = p.value, int(nbytes)

    def tensor(self, shape, dtype, offset: int = 0) -> torch.Tensor:
        n = int(np.prod(shape)) * torch.tensor([], dtype=dtype).element_size()
        if offset + n > self.nbytes:
            raise ValueError('view beyond the buffer')
        owner = self

        class _View:
            __cuda_array_interface__ = {'shape': tuple(int(x) for x in shape), 'typestr': self._typestr[dtype],
                                        'data': (self.ptr + offset, False), 'version': 3, 'strides': None}
            keep = owner
        return torch.as_tensor(_View(), device=torch.device('cuda', torch.cuda.current_device()))

    def __del__(self):
        if getattr(self, 'ptr', None):
            try:
                torch.cuda.synchronize()
                _native.lib().sa_device_free(self.ptr)
            except Exception:
                pass
            self.ptr = None


def _ptr(t: Optional[torch.Tensor]):
    return t.data_ptr() if (t is not None and t.numel()) else None


def features_into(s: _native.SaActions, out: FeatureBlocks, xt_cells: Optional[tuple] = None) -> None:
    """Launch the feature kernels into ``out``. ``xt_cells = (l, w, cells)``: the same pass also
    writes every action's xT cell code for a fit + rate on the (l, w) grid
    (``sa_vaep_features_xt``; ``cells`` from :func:`xt_cells_buffer`)."""
    bb, fb, ib = out.sa_blocks()
    if xt_cells is None:
        _native.check(_native.lib().sa_vaep_features(
            ctypes.byref(s), ctypes.byref(out.plan.struct), ctypes.byref(bb), ctypes.byref(fb),
            ctypes.byref(ib), stream_handle()))
    else:
        l, w, cells = xt_cells
        if cells.dtype != torch.int32 or cells.numel() < s.n:
            raise ValueError('cells must be an int32 tensor of at least n elements')
        _native.check(_native.lib().sa_vaep_features_xt(
            ctypes.byref(s), ctypes.byref(out.plan.struct), ctypes.byref(bb), ctypes.byref(fb),
            ctypes.byref(ib), int(l), int(w), _ptr(cells), stream_handle()))


def features(batch: ActionBatch, xfns: Sequence[str], k: int, flip: bool = True,
             out: Optional[FeatureBlocks] = None, bool_tile: Optional[int] = None,
             num_tile: Optional[int] = None, bool_bits: bool = False,
             num32: bool = False) -> FeatureBlocks:
    """Game-state features of every segment of ``batch`` (windowed mode). ``bool_bits``: the
    bool features as bitmaps (``sa_vaep_features_bits``; 64 instead of 515 B/action written:
    what the staged tree walk of the on-device ``VAEP.rate`` reads). ``num32`` (with
    ``bool_bits``, k <= 3): the numeric blocks in float32 (``sa_vaep_features_bits_f32``: what
    xgboost learners compare; half the numeric bytes written and staged)."""
    plan = out.plan if out is not None else build_plan(xfns, k, batch.atomic)
    if num32 and not bool_bits and out is None:
        raise ValueError('float32 numeric blocks come with the bitmap form (bool_bits=True)')
    if bool_bits and out is None:
        words = max(1, (batch.n + 63) // 64)
        Rn = _ld(batch.n) if num_tile is None else int(num_tile)
        tn = max(1, -(-batch.n // Rn))
        fdt, idt = (torch.float32, torch.float32) if num32 else (torch.float64, torch.int64)
        out = FeatureBlocks(plan, batch.n, 1024, Rn, None,
                            torch.empty((tn, plan.n_f64, Rn), dtype=fdt, device=batch.device),
                            torch.empty((tn, plan.n_i64, Rn), dtype=idt, device=batch.device),
                            torch.empty((max(plan.n_bool, 1), words), dtype=torch.int64,
                                        device=batch.device))
    out = out or alloc_feature_blocks(plan, batch.n, batch.device, bool_tile, num_tile)
    if out.bool_bits is not None and out.bool_block is None:
        _, fb, ib = out.sa_blocks()
        fn = _native.lib().sa_vaep_features_bits_f32 if out.num32 else _native.lib().sa_vaep_features_bits
        _native.check(fn(
            ctypes.byref(batch.struct(flip=flip)), ctypes.byref(out.plan.struct),
            out.bool_bits.data_ptr(), out.bool_bits.shape[1] * 8, max(plan.n_bool, 1),
            ctypes.byref(fb), ctypes.byref(ib), stream_handle()))
        if batch.n % 64:  # the kernel clears rows >= n of the 16-row group holding row n - 1;
            # the last word's later groups are cleared here
            out.bool_bits[:, -1] &= (1 << (batch.n % 64)) - 1
        return out
    features_into(batch.struct(flip=flip), out)
    return out


def features_explicit(frames: Sequence[ActionBatch], xfns: Sequence[str]) -> FeatureBlocks:
    """Features of a user-built list of game-state frames (module-level transformers)."""
    plan = build_plan(xfns, len(frames), frames[0].atomic)
    out = alloc_feature_blocks(plan, frames[0].n, frames[0].device)
    features_into(ActionBatch.explicit_struct(frames), out)
    return out


@dataclass
class LabelBlocks:
    n: int
    scores: torch.Tensor
    concedes: torch.Tensor
    goal_from_shot: torch.Tensor


def labels(batch: ActionBatch, nr_actions: int = 10, out: Optional[LabelBlocks] = None) -> LabelBlocks:
    ld = _ld(batch.n)
    if out is None:
        buf = torch.empty((3, ld), dtype=torch.uint8, device=batch.device)
        out = LabelBlocks(batch.n, buf[0], buf[1], buf[2])
    s = batch.struct()
    _native.check(_native.lib().sa_vaep_labels(ctypes.byref(s), int(nr_actions), _ptr(out.scores),
                                               _ptr(out.concedes), _ptr(out.goal_from_shot), ld,
                                               stream_handle()))
    return out


def formula(batch: ActionBatch, p_scores: torch.Tensor, p_concedes: torch.Tensor,
            out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """offensive / defensive / vaep value as a ``[3, ld]`` tensor of the probability dtype."""
    dt = p_scores.dtype
    if dt not in (torch.float32, torch.float64) or p_concedes.dtype != dt:
        raise TypeError('probabilities must both be float32 or both float64')
    if p_scores.numel() < batch.n or p_concedes.numel() < batch.n:
        raise ValueError('one probability per action is required')
    ps, pc = p_scores.contiguous(), p_concedes.contiguous()
    if out is None:
        out = torch.empty((3, _ld(batch.n)), dtype=dt, device=batch.device)
    s = batch.struct()
    fn = _native.lib().sa_vaep_formula_f64 if dt == torch.float64 else \
        _native.lib().sa_vaep_formula_f32
    _native.check(fn(ctypes.byref(s), _ptr(ps), _ptr(pc), _ptr(out[0]), _ptr(out[1]),
                     _ptr(out[2]), stream_handle()))
    return out


def labels_formula(batch: ActionBatch, p_scores: torch.Tensor, p_concedes: torch.Tensor,
                   nr_actions: int = 10, labels_out: Optional[LabelBlocks] = None,
                   values_out: Optional[torch.Tensor] = None) -> Tuple[LabelBlocks, torch.Tensor]:
    """:func:`labels` and :func:`formula` of the same actions in one launch."""
    dt = p_scores.dtype
    if dt not in (torch.float32, torch.float64) or p_concedes.dtype != dt:
        raise TypeError('probabilities must both be float32 or both float64')
    if p_scores.numel() < batch.n or p_concedes.numel() < batch.n:
        raise ValueError('one probability per action is required')
    ld = _ld(batch.n)
    if labels_out is None:
        buf = torch.empty((3, ld), dtype=torch.uint8, device=batch.device)
        labels_out = LabelBlocks(batch.n, buf[0], buf[1], buf[2])
    if values_out is None:
        values_out = torch.empty((3, ld), dtype=dt, device=batch.device)
    ps, pc = p_scores.contiguous(), p_concedes.contiguous()
    s = batch.struct()
    fn = _native.lib().sa_vaep_labels_formula_f64 if dt == torch.float64 else \
        _native.lib().sa_vaep_labels_formula_f32
    o = values_out
    _native.check(fn(ctypes.byref(s), int(nr_actions), _ptr(labels_out.scores),
                     _ptr(labels_out.concedes), _ptr(labels_out.goal_from_shot), ld, _ptr(ps),
                     _ptr(pc), _ptr(o[0]), _ptr(o[1]), _ptr(o[2]), stream_handle()))
    return labels_out, values_out


def step_into(s: _native.SaActions, out: FeatureBlocks, p_scores: Optional[torch.Tensor],
              p_concedes: Optional[torch.Tensor], nr_actions: int, labels_out: LabelBlocks,
              values_out: Optional[torch.Tensor], xt_cells: Optional[tuple] = None,
              chunk_rows: int = 0, prefetch: bool = False) -> None:
    """The batch valuation step in one call (``sa_vaep_step_f64``): the features of ``out``'s
    plan (and, with ``xt_cells = (l, w, cells)``, every action's xT cell code), the labels and
    the f64 formula of the same actions -- exactly :func:`features_into` followed by
    :func:`labels_formula`, with the labels and formula computed inside the numeric pass.
    ``p_scores = p_concedes = values_out = None``: features + labels only."""
    if p_scores is not None:
        if p_scores.dtype != torch.float64 or p_concedes.dtype != torch.float64:
            raise TypeError('the fused step takes float64 probabilities (float32: labels_formula)')
        if p_scores.numel() < s.n or p_concedes.numel() < s.n:
            raise ValueError('one probability per action is required')
        ps, pc = p_scores.contiguous(), p_concedes.contiguous()
        o = (values_out[0], values_out[1], values_out[2])
    else:  # features + labels only
        ps = pc = None
        o = (None, None, None)
    l, w, cells = xt_cells if xt_cells is not None else (0, 0, None)
    if cells is not None and (cells.dtype != torch.int32 or cells.numel() < s.n):
        raise ValueError('cells must be an int32 tensor of at least n elements')
    bb, fb, ib = out.sa_blocks()
    if chunk_rows:  # A/B probe: the numeric pass in chunks, optionally prefetched (bench --num-chunks)
        _native.check(_native.lib().sa_vaep_step_f64_chunked(
            ctypes.byref(s), ctypes.byref(out.plan.struct), ctypes.byref(bb), ctypes.byref(fb),
            ctypes.byref(ib), int(l), int(w), _ptr(cells), int(nr_actions), _ptr(labels_out.scores),
            _ptr(labels_out.concedes), _ptr(labels_out.goal_from_shot), _ld(s.n), _ptr(ps), _ptr(pc),
            _ptr(o[0]), _ptr(o[1]), _ptr(o[2]), int(chunk_rows), int(prefetch), stream_handle()))
        return
    _native.check(_native.lib().sa_vaep_step_f64(
        ctypes.byref(s), ctypes.byref(out.plan.struct), ctypes.byref(bb), ctypes.byref(fb),
        ctypes.byref(ib), int(l), int(w), _ptr(cells), int(nr_actions), _ptr(labels_out.scores),
        _ptr(labels_out.concedes), _ptr(labels_out.goal_from_shot), _ld(s.n), _ptr(ps), _ptr(pc),
        _ptr(o[0]), _ptr(o[1]), _ptr(o[2]), stream_handle()))


# ------------------------------------------------------------------------------- xT
@dataclass
class XTCounts:
    l: int
    w: int
    shot: torch.Tensor   # int64 [C]
    goal: torch.Tensor   # int64 [C]
    move: torch.Tensor   # int64 [C]
    trans: torch.Tensor  # int32 [C*C]
    err: torch.Tensor    # int32 [1]
    # the transition counts' compact rows (ell, row_len) as the count wrote them for the solve
    # (xt_count_many on 1025 - 9472 cells); every op that changes the counts drops them
    compact: Optional[Tuple[torch.Tensor, torch.Tensor]] = None
    # False: the count wrote the compact rows only (xt_count_buckets(dense=False)): ``trans``
    # holds just the rows of bands with a count >= 65535, the compact rows are the counts
    dense: bool = True

    @property
    def C(self) -> int:
        return self.l * self.w

    def zero_(self) -> 'XTCounts':
        """Zero every count in one fill of the backing buffer (on the current stream)."""
        self.compact = None
        self.dense = True
        self.buf.zero_()
        return self

    def require_dense(self, what: str) -> None:
        if not self.dense:
            raise ValueError(f'{what} reads the dense C x C transition counts, which this count '
                             'did not write (xt_count_buckets(dense=False)); count with dense=True')


def xt_zero_counts(l: int, w: int, dev, row_blocks: int = 1, zero_counts: bool = True) -> XTCounts:
    """Zeroed count buffers, carved from ONE allocation (one fill kernel, one all-reduce):
    ``[shot | goal | move]`` (3 x C int64), the error flags (int32), then the C x C transition
    counts (int32). ``row_blocks`` > 1 pads the transition counts to a whole number of equal row
    blocks (``XTCounts.trans_padded``) so they can be reduce-scattered by rows across that many
    ranks; ``trans`` is the C*C view the count kernel fills. ``XTCounts.head`` is the vectors +
    flags part, ``XTCounts.buf`` the whole allocation. ``zero_counts=False``: only the error
    flags are zeroed (for a count that overwrites every row, ``row_blocks`` 1)."""
    C = l * w
    rows = -(-C // row_blocks) * row_blocks
    a = lambda b: -(-b // 256) * 256  # noqa: E731  (256-B aligned parts)
    o_err = a(3 * C * 8)
    o_tr = o_err + 256
    if zero_counts or row_blocks != 1:
        buf = torch.zeros(o_tr + a(rows * C * 4), dtype=torch.uint8, device=dev)
    else:
        buf = torch.empty(o_tr + a(rows * C * 4), dtype=torch.uint8, device=dev)
        buf[o_err:o_tr].zero_()
    vec = buf[:3 * C * 8].view(torch.int64).view(3, C)
    padded = buf[o_tr:o_tr + rows * C * 4].view(torch.int32)
    acc = XTCounts(l, w, vec[0], vec[1], vec[2], padded[:C * C], buf[o_err:o_err + 4].view(torch.int32))
    acc.trans_padded = padded
    acc.head = buf[:o_tr]
    acc.buf = buf
    return acc


def xt_count(batch: ActionBatch, l: int, w: int, acc: Optional[XTCounts] = None,
             codes: Optional[torch.Tensor] = None, shared: bool = False) -> XTCounts:
    """Count pass of ExpectedThreat.fit. With ``codes`` (u32 [>= n], e.g. from
    :func:`xt_rate_codes_buffer`) the pass also writes each action's rate operand for a later
    :func:`xt_rate_codes` of the same actions on the same grid. ``shared``: the pass runs next
    to other kernels (workgroups sized to co-reside with them)."""
    acc = acc or xt_zero_counts(l, w, batch.device)
    acc.require_dense('adding to a count')
    acc.compact = None  # the counts change
    s = batch.struct()
    if codes is None and not shared:
        _native.check(_native.lib().sa_xt_count(ctypes.byref(s), l, w, _ptr(acc.shot),
                                                _ptr(acc.goal), _ptr(acc.move), _ptr(acc.trans),
                                                _ptr(acc.err), stream_handle()))
    else:
        if codes is not None and (codes.dtype != torch.int32 or codes.numel() < batch.n):
            raise ValueError('codes must be an int32 tensor of at least n elements')
        _native.check(_native.lib().sa_xt_count_codes(ctypes.byref(s), l, w, _ptr(acc.shot),
                                                      _ptr(acc.goal), _ptr(acc.move),
                                                      _ptr(acc.trans), _ptr(acc.err),
                                                      _ptr(codes), int(shared),
                                                      stream_handle()))
    return acc


def xt_band_shape(l: int, w: int) -> Optional[Tuple[int, int]]:
    """(start cells per band, bands) of the band-owned count of an (l, w) grid, or None when
    the grid takes the LDS-histogram (small) or global-atomic (very large) count instead."""
    C = l * w
    if C <= 202 or C > 46340:  # the XC_WIDE / XC_SMALL LDS passes hold these whole
        return None
    r, nb = ctypes.c_int32(0), ctypes.c_int32(0)
    if _native.lib().sa_xt_band_shape(int(l), int(w), ctypes.byref(r), ctypes.byref(nb)) != 0:
        return None
    return r.value, nb.value


@dataclass
class XTBuckets:
    """One batch's counted actions sorted by start-cell band (``sa_xt_count_bucket``)."""
    keys: torch.Tensor      # u16 (as int16) [n]: each key's bin in its band's histogram
    band_off: torch.Tensor  # int64 [n_bands + 1]


def xt_bucket(batch: Optional[ActionBatch], l: int, w: int, err: torch.Tensor,
              cells: Optional[torch.Tensor] = None, n: Optional[int] = None,
              codes: Optional[torch.Tensor] = None,
              interp_codes: Optional[torch.Tensor] = None, L: int = 1050,
              W: int = 680) -> XTBuckets:
    """The per-batch half of the band-owned count: every counted action of ``batch`` (or of
    ``n`` cell codes) as a 4-B key, sorted by start-cell band; error bytes into ``err``.
    ``interp_codes`` (int64 [>= n], :func:`xt_interp_codes_buffer`): each action's operand of a
    later :func:`xt_rate_interp_codes` of the same actions on the L x W node grid."""
    if cells is not None and (codes is not None or interp_codes is not None):
        raise ValueError('rate operands come from the coordinate pass, not from cell codes')
    if cells is None and batch is None:
        raise ValueError('a batch or cell codes are required')
    n = batch.n if cells is None else int(n)
    if interp_codes is not None and (interp_codes.dtype != torch.int64 or
                                     interp_codes.numel() < n):
        raise ValueError('interp_codes must be an int64 tensor of at least n elements')
    if codes is not None and (codes.dtype != torch.int32 or codes.numel() < n):
        raise ValueError('codes must be an int32 tensor of at least n elements')
    shape = xt_band_shape(l, w)
    if shape is None:
        raise ValueError(f'the band-owned count does not take a {l} x {w} grid')
    dev = err.device
    keys = torch.empty(max(n, 16), dtype=torch.int16, device=dev)  # u16 bins (sa_xt_count_bucket)
    off = torch.empty(shape[1] + 1, dtype=torch.int64, device=dev)
    s = batch.struct() if cells is None else None
    _native.check(_native.lib().sa_xt_count_bucket(
        ctypes.byref(s) if s is not None else None, _ptr(cells), int(n), int(l), int(w), _ptr(keys),
        _ptr(off), _ptr(err), _ptr(codes), _ptr(interp_codes), int(L), int(W), stream_handle()))
    return XTBuckets(keys, off)


def xt_interp_codes_buffer(n: int, dev) -> torch.Tensor:
    """u64 interpolated-rate operands (stored as int64) for n actions."""
    return torch.empty(max(_ld(n), 16), dtype=torch.int64, device=dev)


def xt_rate_interp_codes(icodes: torch.Tensor, n: int, xT: torch.Tensor, l: int, w: int,
                         L: int = 1050, W: int = 680, axes: Optional[torch.Tensor] = None,
                         out: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """:func:`xt_rate_interp` of the actions whose bucket pass wrote ``icodes``: the same
    values, NaN pattern and error bit, reading 8 B per action."""
    dev = icodes.device
    axes = xt_interp_axes(l, w, dev, L, W) if axes is None else axes
    if axes.numel() != l + w + L + W:
        raise ValueError('axes must hold l + w + L + W node positions')
    out = torch.empty(max(_ld(n), 16), dtype=torch.float64, device=dev) if out is None else out
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    o = l + w
    _native.check(_native.lib().sa_xt_rate_interp_codes(
        _ptr(icodes), int(n), _ptr(xT.contiguous()), _ptr(axes[:l]), _ptr(axes[l:o]), l, w,
        _ptr(axes[o:o + L]), L, _ptr(axes[o + L:]), W, _ptr(out), _ptr(err), stream_handle()))
    return out[:n], err


def xt_rate_interp_codes_many(icodes: Sequence[torch.Tensor], ns: Sequence[int], xT: torch.Tensor,
                              l: int, w: int, L: int = 1050, W: int = 680,
                              axes: Optional[torch.Tensor] = None,
                              outs: Optional[Sequence[torch.Tensor]] = None
                              ) -> Tuple[List[torch.Tensor], torch.Tensor]:
    """:func:`xt_rate_interp_codes` of several batches (a fit's device batches) in one launch
    (``sa_xt_rate_interp_codes_many``): the same values per batch, one error word for all."""
    if len(icodes) != len(ns) or (outs is not None and len(outs) != len(ns)):
        raise ValueError('one operand buffer, count (and out) per batch')
    dev = xT.device
    axes = xt_interp_axes(l, w, dev, L, W) if axes is None else axes
    if axes.numel() != l + w + L + W:
        raise ValueError('axes must hold l + w + L + W node positions')
    ns = [int(n) for n in ns]
    for c, n in zip(icodes, ns):
        if n < 0 or c.numel() * c.element_size() < 8 * n:
            raise ValueError('an operand buffer holds fewer than n codes')
    outs = [torch.empty(max(_ld(n), 16), dtype=torch.float64, device=dev) for n in ns] \
        if outs is None else list(outs)
    for o, n in zip(outs, ns):
        if o.dtype != torch.float64 or o.numel() < n:
            raise ValueError('out must be float64 with room for n values')
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    k = len(ns)
    cp = (ctypes.c_void_p * max(k, 1))(*[c.data_ptr() for c in icodes])
    op = (ctypes.c_void_p * max(k, 1))(*[o.data_ptr() for o in outs])
    nn = (ctypes.c_int64 * max(k, 1))(*ns)
    o = l + w
    _native.check(_native.lib().sa_xt_rate_interp_codes_many(
        k, cp, nn, _ptr(xT.contiguous()), _ptr(axes[:l]), _ptr(axes[l:o]), l, w,
        _ptr(axes[o:o + L]), L, _ptr(axes[o + L:]), W, op, _ptr(err), stream_handle()))
    return [t[:n] for t, n in zip(outs, ns)], err


def xt_fit_rate_interp_codes(acc: XTCounts, icodes: Sequence[torch.Tensor], ns: Sequence[int],
                             L: int = 1050, W: int = 680, axes: Optional[torch.Tensor] = None,
                             outs: Optional[Sequence[torch.Tensor]] = None, eps: float = 1e-5,
                             max_iter: int = 1000, exact_order: bool = False
                             ) -> Tuple[XTSolution, List[torch.Tensor], torch.Tensor]:
    """:func:`xt_solve` (``transition=False``) then :func:`xt_rate_interp_codes_many` over the
    surface, in one call (``sa_xt_fit_rate_interp_codes``, grids above ``SA_XT_SOLVE_MAX_C``
    cells): the rate is queued right behind the one-launch solve instead of after its host
    round trip.  The same outputs as the two calls."""
    C, l, w = acc.C, acc.l, acc.w
    if C <= _native.SA_XT_SOLVE_MAX_C:
        raise ValueError('the fused fit + rate is for grids above SA_XT_SOLVE_MAX_C cells')
    if len(icodes) != len(ns) or (outs is not None and len(outs) != len(ns)):
        raise ValueError('one operand buffer, count (and out) per batch')
    if getattr(acc, 'compact', None) is None:
        acc.require_dense('xt_fit_rate_interp_codes without compact rows')
    dev = acc.shot.device
    axes = xt_interp_axes(l, w, dev, L, W) if axes is None else axes
    if axes.numel() != l + w + L + W:
        raise ValueError('axes must hold l + w + L + W node positions')
    ns = [int(n) for n in ns]
    for c, n in zip(icodes, ns):
        if n < 0 or c.numel() * c.element_size() < 8 * n:
            raise ValueError('an operand buffer holds fewer than n codes')
    outs = [torch.empty(max(_ld(n), 16), dtype=torch.float64, device=dev) for n in ns] \
        if outs is None else list(outs)
    for o, n in zip(outs, ns):
        if o.dtype != torch.float64 or o.numel() < n:
            raise ValueError('out must be float64 with room for n values')
    mats = torch.empty((4, C), dtype=torch.float64, device=dev)
    heat = torch.empty((max_iter + 1, C), dtype=torch.float64, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    k = len(ns)
    cp = (ctypes.c_void_p * max(k, 1))(*[c.data_ptr() for c in icodes])
    op = (ctypes.c_void_p * max(k, 1))(*[o.data_ptr() for o in outs])
    nn = (ctypes.c_int64 * max(k, 1))(*ns)
    n_iter, path = ctypes.c_int32(0), ctypes.c_int32(0)
    ell, rl = acc.compact if getattr(acc, 'compact', None) is not None else (None, None)
    o = l + w
    _native.check(_native.lib().sa_xt_fit_rate_interp_codes(
        _ptr(acc.shot), _ptr(acc.goal), _ptr(acc.move), _ptr(acc.trans), l, w, float(eps),
        int(max_iter), _native.SA_XT_SOLVE_EXACT if exact_order else 0, _ptr(mats), _ptr(heat),
        ctypes.byref(n_iter), ctypes.byref(path), _ptr(ell), _ptr(rl), k, cp, nn, _ptr(axes[:l]),
        _ptr(axes[l:o]), _ptr(axes[o:o + L]), L, _ptr(axes[o + L:]), W, op, _ptr(err), stream_handle()))
    if n_iter.value < 0:
        raise RuntimeError(f'xT value iteration did not converge within {max_iter} iterations')
    p = _native.XT_SOLVE_PATHS[path.value]
    _warn_solve_path(p)
    sol = XTSolution(mats, None, heat[:n_iter.value + 1], n_iter.value, p)
    return sol, [t[:n] for t, n in zip(outs, ns)], err


XB_MAX_SETS = 24  # bucket sets one band-count launch takes (sa_xt_large.hip)


def _compact_pitch(C: int) -> int:
    return int(_native.lib().sa_xt_compact_bytes(C, 1)) // 4


def xt_count_buckets(parts: Sequence[XTBuckets], l: int, w: int, acc: XTCounts,
                     overwrite: bool = False, compact: Optional[bool] = None,
                     dense: bool = True) -> XTCounts:
    """The once-per-fit half of the band-owned count: every batch's buckets into ``acc`` (added;
    ``overwrite``: written, the rows' old values never read).  ``compact`` (default: whenever it
    can) also writes the transition counts' compact rows for the large-grid solve
    (``sa_xt_count_from_buckets_ex``; ``acc.compact``): overwrite, <= 24 batches and
    1025 <= C <= 9472 only.  ``dense=False`` (with the compact rows): the dense C x C table is
    not written (``SA_XT_COUNT_COMPACT_ONLY``: only the rows of bands holding a count >= 65535,
    which the compact solve reads) -- for a fit that reads the compact rows alone (the solve,
    :func:`xt_transition_entries`); ``acc.dense`` is then False."""
    k = len(parts)
    C = l * w
    can = (overwrite and k <= XB_MAX_SETS and _native.SA_XT_SOLVE_MAX_C < C <= _native.SA_XT_COMPACT_MAX_C)
    if compact and not can:
        raise ValueError('compact rows need overwrite, at most 24 batches and 1025 <= C <= 9472')
    compact = can if compact is None else compact
    dense = dense or not compact  # the dense rows are skipped only beside the compact rows
    acc.compact = None
    acc.dense = True
    ell = rl = None
    if compact:
        pe = _compact_pitch(C)
        ell = torch.empty(C * pe, dtype=torch.int32, device=acc.trans.device)
        rl = torch.empty(C, dtype=torch.int32, device=acc.trans.device)
    keys = (ctypes.c_void_p * max(k, 1))(*[p.keys.data_ptr() for p in parts])
    offs = (ctypes.c_void_p * max(k, 1))(*[p.band_off.data_ptr() for p in parts])
    flags = (_native.SA_XT_COUNT_OVERWRITE if overwrite else 0) | \
        (0 if dense else _native.SA_XT_COUNT_COMPACT_ONLY)
    _native.check(_native.lib().sa_xt_count_from_buckets_ex(
        k, keys, offs, int(l), int(w), _ptr(acc.shot), _ptr(acc.goal), _ptr(acc.move),
        _ptr(acc.trans), flags, _ptr(ell), _ptr(rl), stream_handle()))
    if compact:
        acc.compact = (ell, rl)
    acc.dense = dense
    return acc


def xt_transition_entries(acc: XTCounts) -> Tuple[torch.Tensor, torch.Tensor]:
    """The non-zero transition counts as ``(flat index s * C + e, count)`` int64 device tensors
    in row-major order -- from the compact rows when the count wrote them (62.5 MB read at
    105 x 68; counts >= 65535 from their dense rows), else from the dense table."""
    C = acc.shot.numel()
    if getattr(acc, 'compact', None) is None:
        if not getattr(acc, 'dense', True):
            acc.require_dense('xt_transition_entries without compact rows')
        nz = torch.nonzero(acc.trans).reshape(-1)
        return nz, acc.trans[nz].to(torch.int64)
    ell, rl = acc.compact
    pe = ell.numel() // C
    k = torch.arange(pe, device=ell.device)
    # storage slot of a row's k-th entry (sa_xt_large.hip xe_slot)
    slot = (k & ~127) | ((k & 31) << 2) | ((k >> 5) & 3)
    e = ell.view(C, pe)[:, slot].to(torch.int64) & 0xFFFFFFFF  # [C, pe], entry k of each row
    used = k.unsqueeze(0) < rl.to(torch.int64).unsqueeze(1)
    rows = torch.arange(C, device=ell.device).unsqueeze(1).expand(C, pe)[used]
    e = e[used]
    idx = rows * C + (e & 0xFFFF)
    cnt = e >> 16
    esc = cnt == 0xFFFF  # escaped: the dense row holds the count (written for its band)
    if bool(esc.any()):
        cnt = torch.where(esc, acc.trans[idx].to(torch.int64), cnt)
    return idx, cnt


def xt_count_many(batches: Sequence[ActionBatch], l: int, w: int,
                  acc: Optional[XTCounts] = None, overwrite: Optional[bool] = None,
                  interp_codes: Optional[Sequence[torch.Tensor]] = None,
                  dense: bool = True) -> XTCounts:
    """The count pass of ONE fit over several device batches (e.g. cfg5's 1e8 actions in
    batches of <= 10k games): equal to :func:`xt_count` of every batch into one accumulator.
    Band-owned grids bucket each batch and write the C x C table once. ``overwrite`` (default:
    ``acc`` is None, a fresh accumulator): the counts are written, not added to the old ones
    (``acc``'s error flags still accumulate). ``interp_codes``: one :func:`xt_interp_codes_buffer`
    per batch (band-owned grids only), filled for a later :func:`xt_rate_interp_codes`.
    ``dense=False``: see :func:`xt_count_buckets` (band-owned grids with compact rows only;
    ignored elsewhere)."""
    if xt_band_shape(l, w) is None or not batches:
        if interp_codes is not None:
            raise ValueError('interp_codes come from the band-owned count')
        if overwrite and acc is not None:  # the counts only: the error flags accumulate, as on
            for t in (acc.shot, acc.goal, acc.move, acc.trans):  # the band-owned path
                t.zero_()
            acc.compact = None  # they described the old counts
            acc.dense = True
        if acc is not None and not acc.dense:  # adding to rows that were never written
            acc.require_dense('adding to a count')
        for b in batches:
            acc = xt_count(b, l, w, acc)
        return acc if acc is not None else xt_zero_counts(l, w, torch.device('cuda'))
    if overwrite is None:
        overwrite = acc is None
    if acc is not None and not acc.dense and not overwrite:
        acc.require_dense('adding to a count')
    # a fresh accumulator the overwriting count fills whole: only its error word zeroed (the
    # 204 MB fill of the 105 x 68 table was 27 us of cfg5's fit)
    acc = acc or xt_zero_counts(l, w, batches[0].device, zero_counts=not overwrite)
    ic = list(interp_codes) if interp_codes is not None else [None] * len(batches)
    parts = [xt_bucket(b, l, w, acc.err, interp_codes=c) for b, c in zip(batches, ic)]
    return xt_count_buckets(parts, l, w, acc, overwrite=overwrite, dense=dense)


def xt_rate_codes_buffer(n: int, dev) -> torch.Tensor:
    """u32 rate operands (stored as int32) for n actions."""
    return torch.empty(max(_ld(n), 16), dtype=torch.int32, device=dev)


def xt_rate_codes(codes: torch.Tensor, n: int, grid: torch.Tensor,
                  out: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """ExpectedThreat.rate (no interpolation) of the actions whose count pass wrote ``codes``,
    ``grid`` = the fitted (w, l) surface: same values and error bit as :func:`xt_rate`."""
    dev = codes.device
    out = torch.empty(max(_ld(n), 16), dtype=torch.float64, device=dev) if out is None else out
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    _native.check(_native.lib().sa_xt_rate_codes(_ptr(codes), n, _ptr(grid.contiguous()),
                                                 _ptr(out), _ptr(err), stream_handle()))
    return out[:n], err


# the count pass's error flags, one BYTE each (sa_xt_count: 0x1 / 0x100 / 0x10000 per rank), so
# the flags of up to 255 ranks add up in the counts' one sum all-reduce without carrying into
# each other; a flag is set when its byte is non-zero
XT_ERR_SHOT, XT_ERR_MOVE_START, XT_ERR_MOVE_OTHER = 0xFF, 0xFF00, 0xFF0000
# a rank's counts too large for the multi-GPU int32-word sum (shard.allreduce_xt_counts)
XT_ERR_OVERFLOW = 0xFF000000
XT_ERR_FIT = XT_ERR_SHOT | XT_ERR_MOVE_START | XT_ERR_MOVE_OTHER | XT_ERR_OVERFLOW


def xt_cells_buffer(n: int, dev) -> torch.Tensor:
    """u32 xT cell codes (stored as int32) for n actions."""
    return torch.empty(max(_ld(n), 16), dtype=torch.int32, device=dev)


def xt_cell_codes(cells: torch.Tensor, n: int, l: int, w: int) -> torch.Tensor:
    """The n meaningful codes of a cell-code buffer: int16 (the 16-bit codes of grids of <=
    SA_XT_CELLS16_MAX_C cells) or int32."""
    if l * w <= _native.SA_XT_CELLS16_MAX_C:
        return cells.view(torch.int16)[:n]
    return cells[:n]


def xt_cells(batch: ActionBatch, l: int, w: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """The xT cell code of every action (``sa_xt_cells``: the count pass's binning alone)."""
    out = xt_cells_buffer(batch.n, batch.device) if out is None else out
    s = batch.struct()
    _native.check(_native.lib().sa_xt_cells(ctypes.byref(s), int(l), int(w), _ptr(out),
                                            stream_handle()))
    return out


def xt_count_cells(cells: torch.Tensor, n: int, l: int, w: int, acc: Optional[XTCounts] = None,
                   shared: bool = False) -> XTCounts:
    """The count pass of ExpectedThreat.fit from cell codes (4 B per action read)."""
    acc = acc or xt_zero_counts(l, w, cells.device)
    acc.require_dense('adding to a count')
    acc.compact = None  # the counts change
    _native.check(_native.lib().sa_xt_count_cells(_ptr(cells), int(n), int(l), int(w),
                                                  _ptr(acc.shot), _ptr(acc.goal), _ptr(acc.move),
                                                  _ptr(acc.trans), _ptr(acc.err), int(shared),
                                                  stream_handle()))
    return acc


def xt_rate_cells(cells: torch.Tensor, n: int, l: int, w: int, grid: torch.Tensor,
                  out: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """ExpectedThreat.rate (no interpolation, grid = the (w, l) surface) from cell codes."""
    dev = cells.device
    out = torch.empty(max(_ld(n), 16), dtype=torch.float64, device=dev) if out is None else out
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    _native.check(_native.lib().sa_xt_rate_cells(_ptr(cells), int(n), int(l), int(w),
                                                 _ptr(grid.contiguous()), _ptr(out), _ptr(err),
                                                 stream_handle()))
    return out[:n], err


def xt_check_errors(acc: XTCounts, mask: int = XT_ERR_FIT) -> None:
    """Raise where the reference's int64 cast raises. ``mask`` selects what the caller reads:
    shots (scoring_prob), shots and move starts (action_prob), every move coordinate
    (move_transition_matrix) or everything (fit)."""
    e = int(acc.err.item()) & mask
    if e & XT_ERR_OVERFLOW:
        raise OverflowError('xT counts of one rank reach 2**31 / world: the multi-GPU count sum '
                            'would overflow its int32 words')
    if e & XT_ERR_MOVE_OTHER:
        raise ValueError('Cannot convert non-finite values (NA or inf) to integer '
                         '(move coordinates)')
    if e & XT_ERR_SHOT:
        raise ValueError('Cannot convert non-finite values (NA or inf) to integer '
                         '(shot start coordinates)')
    if e & XT_ERR_MOVE_START:
        raise ValueError('Cannot convert non-finite values (NA or inf) to integer '
                         '(move coordinates)')


@dataclass
class XTSolution:
    mats: torch.Tensor      # f64 [4, C]: scoring, shot, move, xT
    trans_t: Optional[torch.Tensor]  # f64 [C, C] transposed transition matrix (or None)
    heatmaps: torch.Tensor  # f64 [n_iter + 1, C]
    n_iter: int
    path: str = 'sequential'  # _native.XT_SOLVE_PATHS: how the value iteration summed its rows


def xt_solve(acc: XTCounts, eps: float = 1e-5, max_iter: int = 1000,
             transition: bool = True, exact_order: bool = False) -> XTSolution:
    """Normalisation + value iteration. ``transition=False`` (grids above
    ``SA_XT_SOLVE_MAX_C`` cells only) skips forming the dense transposed transition matrix,
    which the large-grid iteration never reads (408 MB at 105 x 68).  Grids above
    ``SA_XT_SOLVE_MAX_C`` cells sum each row in a fixed parallel order under an error bound that
    keeps every convergence decision, and so the iteration count, the reference's (iterates
    within 4e-11 relative at 105 x 68; ``sa_xt_solve_ex``); ``exact_order=True`` sums in the
    reference's order (bit-exact iterates).  ``XTSolution.path`` says which ran."""
    C = acc.C
    dev = acc.shot.device
    mats = torch.empty((4, C), dtype=torch.float64, device=dev)
    if not transition and C <= _native.SA_XT_SOLVE_MAX_C:
        transition = True  # the small-grid solve reads the transposed matrix
    if transition or getattr(acc, 'compact', None) is None:
        acc.require_dense('xt_solve with the transition matrix or without compact rows')
    tt = torch.empty((C, C), dtype=torch.float64, device=dev) if transition else None
    heat = torch.empty((max_iter + 1, C), dtype=torch.float64, device=dev)
    n_iter, path = ctypes.c_int32(0), ctypes.c_int32(0)
    ell, rl = acc.compact if getattr(acc, 'compact', None) is not None else (None, None)
    _native.check(_native.lib().sa_xt_solve_ex(
        _ptr(acc.shot), _ptr(acc.goal), _ptr(acc.move), _ptr(acc.trans), acc.l, acc.w, float(eps),
        int(max_iter), _native.SA_XT_SOLVE_EXACT if exact_order else 0, _ptr(mats), _ptr(tt),
        _ptr(heat), ctypes.byref(n_iter), ctypes.byref(path), _ptr(ell), _ptr(rl),
        stream_handle()))
    if n_iter.value < 0:
        raise RuntimeError(f'xT value iteration did not converge within {max_iter} iterations')
    p = _native.XT_SOLVE_PATHS[path.value]
    _warn_solve_path(p)
    return XTSolution(mats, tt, heat[:n_iter.value + 1], n_iter.value, p)


def _warn_solve_path(path: str) -> None:
    if path == 'timeout':
        import warnings
        warnings.warn('the reordered xT solve timed out at a grid barrier (another kernel held '
                      'CUs: it needs one workgroup resident on every CU) and was redone in the '
                      "reference's order: same result, ~50 ms - 1 s slower", RuntimeWarning,
                      stacklevel=3)


def xt_solve_compact(ell: torch.Tensor, row_len: torch.Tensor, cnt_rows: torch.Tensor,
                     move: torch.Tensor, gs: torch.Tensor, pmove: torch.Tensor, C: int,
                     eps: float = 1e-5, max_iter: int = 1000,
                     exact_order: bool = False) -> Tuple[torch.Tensor, int, str]:
    """The whole value iteration from the compact form of every row (``sa_xt_solve_compact``):
    ``(heatmaps [max_iter + 1, C] (rows past n_iter unused), n_iter, path)``."""
    heat = torch.empty((max_iter + 1, C), dtype=torch.float64, device=ell.device)
    n_iter, path = ctypes.c_int32(0), ctypes.c_int32(0)
    _native.check(_native.lib().sa_xt_solve_compact(
        _ptr(ell), _ptr(row_len), _ptr(cnt_rows), _ptr(move), _ptr(gs), _ptr(pmove), int(C),
        float(eps), int(max_iter), _native.SA_XT_SOLVE_EXACT if exact_order else 0, _ptr(heat),
        ctypes.byref(n_iter), ctypes.byref(path), stream_handle()))
    p = _native.XT_SOLVE_PATHS[path.value]
    _warn_solve_path(p)
    return heat, n_iter.value, p


def xt_solve_async(acc: XTCounts, eps: float = 1e-5, max_iter: int = 1000) -> XTSolution:
    """:func:`xt_solve` for grids of <= SA_XT_SOLVE_MAX_C cells without the host round trip
    (``sa_xt_solve_async``): ``n_iter`` is a device int32 tensor and the heatmaps are the whole
    ``[max_iter + 1, C]`` buffer; read ``n_iter`` (and check it is >= 0) after synchronising."""
    C = acc.C
    dev = acc.shot.device
    mats = torch.empty((4, C), dtype=torch.float64, device=dev)
    tt = torch.empty((C, C), dtype=torch.float64, device=dev)
    heat = torch.empty((max_iter + 1, C), dtype=torch.float64, device=dev)
    n_iter = torch.empty(1, dtype=torch.int32, device=dev)
    _native.check(_native.lib().sa_xt_solve_async(_ptr(acc.shot), _ptr(acc.goal), _ptr(acc.move),
                                                  _ptr(acc.trans), acc.l, acc.w, float(eps),
                                                  int(max_iter), _ptr(mats), _ptr(tt), _ptr(heat),
                                                  _ptr(n_iter), stream_handle()))
    return XTSolution(mats, tt, heat, n_iter)


def _centres(extent: float, cells: int) -> np.ndarray:
    """Cell centres exactly as the reference (xthreat.py:372-376)."""
    size = extent / cells
    return np.arange(0.0, extent, size) + 0.5 * size


def xt_interp_grid(xT: torch.Tensor, l: int, w: int, xs: Optional[np.ndarray] = None,
                   ys: Optional[np.ndarray] = None, L: int = 1050, W: int = 680,
                   cx: Optional[np.ndarray] = None, cy: Optional[np.ndarray] = None) -> torch.Tensor:
    """Bilinear xT surface on the nodes xs x ys (default: the reference's 1050 x 680
    ``linspace`` grid of ExpectedThreat.rate, xthreat.py:443-451) as a ``[W, L]`` tensor.
    ``cx`` / ``cy``: the surface's node positions (default: the cell centres of
    xthreat.py:372-376), strictly increasing."""
    cx = _centres(105.0, l) if cx is None else np.asarray(cx, np.float64).reshape(-1)
    cy = _centres(68.0, w) if cy is None else np.asarray(cy, np.float64).reshape(-1)
    if len(cx) != l or len(cy) != w:
        raise ValueError('x and y must have the lengths of the xT surface')  # interp2d would
    if (np.diff(cx) <= 0).any() or (np.diff(cy) <= 0).any() or \
            not (np.isfinite(cx).all() and np.isfinite(cy).all()):
        raise ValueError('x and y must be finite and strictly increasing')
    if xs is None:
        xs = np.linspace(0, 105.0, L)
    if ys is None:
        ys = np.linspace(0, 68.0, W)
    xs = np.sort(np.asarray(xs, np.float64).reshape(-1))
    ys = np.sort(np.asarray(ys, np.float64).reshape(-1))
    L, W = len(xs), len(ys)
    dev = xT.device
    c = torch.from_numpy(np.concatenate([cx, cy, xs, ys])).to(dev)
    grid = torch.empty((W, L), dtype=torch.float64, device=dev)
    o = l + w
    _native.check(_native.lib().sa_xt_interp_grid(_ptr(xT.contiguous()), _ptr(c[:l]), _ptr(c[l:o]),
                                                  l, w, _ptr(c[o:o + L]), L, _ptr(c[o + L:]), W,
                                                  _ptr(grid), stream_handle()))
    return grid


def xt_normalize(acc: XTCounts) -> Tuple[torch.Tensor, torch.Tensor]:
    """(mats [3, C] scoring/shot/move probabilities, trans_t [C, C]) on device."""
    acc.require_dense('xt_normalize')
    C = acc.C
    dev = acc.shot.device
    mats = torch.empty((3, C), dtype=torch.float64, device=dev)
    tt = torch.empty((C, C), dtype=torch.float64, device=dev)
    _native.check(_native.lib().sa_xt_normalize(_ptr(acc.shot), _ptr(acc.goal), _ptr(acc.move),
                                                _ptr(acc.trans), acc.l, acc.w, _ptr(mats), _ptr(tt),
                                                stream_handle()))
    return mats, tt


def xt_interp_axes(l: int, w: int, dev, L: int = 1050, W: int = 680) -> torch.Tensor:
    """The node positions of the interpolated rate on the device, ``[cx | cy | xs | ys]``: the
    cell centres (xthreat.py:372-376) and the reference's ``linspace`` nodes (:443-451)."""
    cx, cy = _centres(105.0, l), _centres(68.0, w)
    if len(cx) != l or len(cy) != w:
        raise ValueError('x and y must have the lengths of the xT surface')  # as interp2d
    c = np.concatenate([cx, cy, np.linspace(0, 105.0, L), np.linspace(0, 68.0, W)])
    return torch.from_numpy(c).to(dev)


def xt_rate_interp(batch: ActionBatch, xT: torch.Tensor, l: int, w: int, L: int = 1050,
                   W: int = 680, axes: Optional[torch.Tensor] = None,
                   out: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """ExpectedThreat.rate(use_interpolation=True) of ``batch`` from the (w, l) surface ``xT``
    without the L x W grid (``sa_xt_rate_interp``): bit-identical to
    ``xt_rate(batch, xt_interp_grid(xT, l, w, L=L, W=W), L, W)``. ``axes``: a cached
    :func:`xt_interp_axes` tensor."""
    dev = batch.device
    axes = xt_interp_axes(l, w, dev, L, W) if axes is None else axes
    if axes.numel() != l + w + L + W:
        raise ValueError('axes must hold l + w + L + W node positions')
    out = torch.empty(max(_ld(batch.n), 16), dtype=torch.float64, device=dev) if out is None else out
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    s = batch.struct()
    o = l + w
    _native.check(_native.lib().sa_xt_rate_interp(
        ctypes.byref(s), _ptr(xT.contiguous()), _ptr(axes[:l]), _ptr(axes[l:o]), l, w,
        _ptr(axes[o:o + L]), L, _ptr(axes[o + L:]), W, _ptr(out), _ptr(err), stream_handle()))
    return out[:batch.n], err


def xt_rate(batch: ActionBatch, grid: torch.Tensor, L: int, W: int) -> Tuple[torch.Tensor, torch.Tensor]:
    out = torch.empty(max(batch.n, 1), dtype=torch.float64, device=batch.device)
    err = torch.zeros(1, dtype=torch.int32, device=batch.device)
    s = batch.struct()
    _native.check(_native.lib().sa_xt_rate(ctypes.byref(s), _ptr(grid.contiguous()), L, W,
                                           _ptr(out), _ptr(err), stream_handle()))
    return out[:batch.n], err


def goalscore_into(batch: ActionBatch, out: FeatureBlocks) -> None:
    """Launch only the goalscore scan into the plan's goalscore columns."""
    from ._native import XFN
    gc = out.plan.struct.i64_col[XFN['goalscore']]
    if gc < 0:
        raise ValueError('plan has no goalscore columns')
    s = batch.struct()
    ib = out.sa_blocks()[2]
    _native.check(_native.lib().sa_vaep_goalscore(ctypes.byref(s), ctypes.byref(ib), gc,
                                                  stream_handle()))
