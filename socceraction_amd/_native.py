"""ctypes binding of ``libsocceraction_amd.so`` (the C ABI in ``include/socceraction_amd.h``).

This module is the *only* way the Python layer reaches the HIP kernels. There is no
CPU fallback: if the shared library is missing or no ROCm GPU is visible, every
compute entry point raises. The library is built in-tree by
``python -m socceraction_amd.build`` (or ``__graft_entry__.build()``).
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

HERE = os.path.dirname(os.path.abspath(__file__))
# SOCCERACTION_AMD_DEBUG=1 selects the debug build (device bounds checks, every call checked);
# SOCCERACTION_AMD_LIB an explicit library file (A/B variants)
DEBUG = os.environ.get('SOCCERACTION_AMD_DEBUG', '') not in ('', '0')
DEFAULT_LIB = os.path.join(HERE, '_lib', 'libsocceraction_amd.so')
DEBUG_LIB = os.path.join(HERE, '_lib', 'libsocceraction_amd_debug.so')
LIB_PATH = os.environ.get('SOCCERACTION_AMD_LIB') or (DEBUG_LIB if DEBUG else DEFAULT_LIB)

SA_MAX_FRAMES = 8
SA_SEG_BLOCK = 128  # rows per entry of sa_actions.seg_of_block
SA_XT_SOLVE_MAX_C = 1024  # sa_xt_solve: larger grids may pass trans_t = NULL
SA_XT_CELLS_MAX_C = 4096
SA_XT_COUNT_SHARED, SA_XT_COUNT_OVERWRITE, SA_XT_COUNT_COMPACT_ONLY = 1, 2, 4
SA_XT_CELLS16_MAX_C = 202  # xT cell codes: 16 bits per action up to this many cells
SA_XT_COMPACT_MAX_C = 9472  # sa_xt_compact_rows / sa_xt_iterate_compact
SA_XT_SOLVE_EXACT = 1  # sa_xt_solve_ex / sa_xt_solve_compact: the reference's summation order
# which path produced a large-grid solve (sa_xt_solve_ex's *path)
XT_SOLVE_PATHS = ('sequential', 'reordered', 'inside-bound', 'unavailable', 'timeout')
SA_BOOL_TILE_QUANTUM = 1024
SA_NUM_TILE_QUANTUM = 128
SA_OK, SA_EINVAL, SA_EHIP, SA_EDATA, SA_ENOMEM = 0, -1, -2, -3, -4

# enum sa_xfn (order matters: mirrors include/socceraction_amd.h)
XFN_NAMES = [
    'actiontype', 'actiontype_onehot', 'result', 'result_onehot', 'actiontype_result_onehot',
    'bodypart', 'bodypart_onehot', 'time', 'startlocation', 'endlocation', 'startpolar',
    'endpolar', 'movement', 'team', 'time_delta', 'space_delta', 'goalscore', 'location',
    'polar', 'movement_polar', 'direction',
]
XFN = {name: i for i, name in enumerate(XFN_NAMES)}
SA_XFN_COUNT = len(XFN_NAMES)

_p = ctypes.c_void_p


class SaFrame(ctypes.Structure):
    _fields_ = [('c0', _p), ('c1', _p), ('c2', _p), ('c3', _p), ('time_seconds', _p),
                ('type_id', _p), ('result_id', _p), ('bodypart_id', _p), ('period_id', _p),
                ('team', _p)]


class SaActions(ctypes.Structure):
    _fields_ = [('n', ctypes.c_int64), ('n_segments', ctypes.c_int64), ('seg_off', _p),
                ('home_team', _p), ('n_frames', ctypes.c_int32), ('atomic', ctypes.c_int32),
                ('frames', SaFrame * SA_MAX_FRAMES), ('seg_of_block', _p)]


class SaFeaturePlan(ctypes.Structure):
    _fields_ = [('nb_prev_actions', ctypes.c_int32),
                ('bool_col', ctypes.c_int32 * SA_XFN_COUNT),
                ('f64_col', ctypes.c_int32 * SA_XFN_COUNT),
                ('i64_col', ctypes.c_int32 * SA_XFN_COUNT)]


class SaBlock(ctypes.Structure):
    _fields_ = [('data', _p), ('n_cols', ctypes.c_int32), ('reserved', ctypes.c_int32),
                ('tile_rows', ctypes.c_int64)]


class SaTreeModel(ctypes.Structure):
    _fields_ = [('nodes', ctypes.c_void_p), ('leaf', ctypes.c_void_p), ('roots', ctypes.c_void_p),
                ('tree_depth', ctypes.c_void_p), ('n_nodes', ctypes.c_int32),
                ('n_trees', ctypes.c_int32), ('base_margin', ctypes.c_double),
                ('p_out', ctypes.c_void_p)]


class SaSpadlFrame(ctypes.Structure):
    _fields_ = [('n', ctypes.c_int64), ('time_seconds', _p), ('start_x', _p), ('start_y', _p),
                ('end_x', _p), ('end_y', _p), ('game', _p), ('team', _p), ('player', _p),
                ('event', _p), ('period_id', _p), ('type_id', _p), ('result_id', _p),
                ('bodypart_id', _p), ('order', _p)]


class SaAtomicFrame(ctypes.Structure):
    _fields_ = [('time_seconds', _p), ('x', _p), ('y', _p), ('dx', _p), ('dy', _p),
                ('game', _p), ('team', _p), ('player', _p), ('event', _p), ('period_id', _p),
                ('type_id', _p), ('bodypart_id', _p)]


class SaSpadlOut(ctypes.Structure):
    _fields_ = [('time_seconds', _p), ('start_x', _p), ('start_y', _p), ('end_x', _p),
                ('end_y', _p), ('game', _p), ('team', _p), ('player', _p), ('event', _p),
                ('period_id', _p), ('type_id', _p), ('result_id', _p), ('bodypart_id', _p),
                ('src', _p)]


# name -> (restype, argtypes)
_SIGNATURES = {
    'sa_vaep_features': (ctypes.c_int, [ctypes.POINTER(SaActions), ctypes.POINTER(SaFeaturePlan),
                                        ctypes.POINTER(SaBlock), ctypes.POINTER(SaBlock),
                                        ctypes.POINTER(SaBlock), _p]),
    'sa_vaep_goalscore': (ctypes.c_int, [ctypes.POINTER(SaActions), ctypes.POINTER(SaBlock),
                                         ctypes.c_int32, _p]),
    'sa_vaep_labels': (ctypes.c_int, [ctypes.POINTER(SaActions), ctypes.c_int32, _p, _p, _p,
                                      ctypes.c_int64, _p]),
    'sa_vaep_formula_f64': (ctypes.c_int, [ctypes.POINTER(SaActions), _p, _p, _p, _p, _p, _p]),
    'sa_vaep_formula_f32': (ctypes.c_int, [ctypes.POINTER(SaActions), _p, _p, _p, _p, _p, _p]),
    'sa_vaep_labels_formula_f64': (ctypes.c_int, [ctypes.POINTER(SaActions), ctypes.c_int32, _p, _p,
                                                  _p, ctypes.c_int64, _p, _p, _p, _p, _p, _p]),
    'sa_vaep_labels_formula_f32': (ctypes.c_int, [ctypes.POINTER(SaActions), ctypes.c_int32, _p, _p,
                                                  _p, ctypes.c_int64, _p, _p, _p, _p, _p, _p]),
    'sa_vaep_step_f64': (ctypes.c_int, [ctypes.POINTER(SaActions), ctypes.POINTER(SaFeaturePlan),
                                        ctypes.POINTER(SaBlock), ctypes.POINTER(SaBlock),
                                        ctypes.POINTER(SaBlock), ctypes.c_int32, ctypes.c_int32, _p,
                                        ctypes.c_int32, _p, _p, _p, ctypes.c_int64, _p, _p, _p, _p,
                                        _p, _p]),
    'sa_vaep_step_f64_chunked': (ctypes.c_int, [ctypes.POINTER(SaActions), ctypes.POINTER(SaFeaturePlan),
                                                ctypes.POINTER(SaBlock), ctypes.POINTER(SaBlock),
                                                ctypes.POINTER(SaBlock), ctypes.c_int32, ctypes.c_int32, _p,
                                                ctypes.c_int32, _p, _p, _p, ctypes.c_int64, _p, _p, _p, _p,
                                                _p, ctypes.c_int64, ctypes.c_int32, _p]),
    'sa_xt_count': (ctypes.c_int, [ctypes.POINTER(SaActions), ctypes.c_int32, ctypes.c_int32,
                                   _p, _p, _p, _p, _p, _p]),
    'sa_xt_count_codes': (ctypes.c_int, [ctypes.POINTER(SaActions), ctypes.c_int32,
                                         ctypes.c_int32, _p, _p, _p, _p, _p, _p,
                                         ctypes.c_int32, _p]),
    'sa_xt_rate_codes': (ctypes.c_int, [_p, ctypes.c_int64, _p, _p, _p, _p]),
    'sa_vaep_features_bits': (ctypes.c_int, [ctypes.POINTER(SaActions), ctypes.POINTER(SaFeaturePlan),
                                             _p, ctypes.c_int64, ctypes.c_int32, ctypes.POINTER(SaBlock),
                                             ctypes.POINTER(SaBlock), _p]),
    'sa_vaep_features_bits_f32': (ctypes.c_int, [ctypes.POINTER(SaActions), ctypes.POINTER(SaFeaturePlan),
                                                 _p, ctypes.c_int64, ctypes.c_int32, ctypes.POINTER(SaBlock),
                                                 ctypes.POINTER(SaBlock), _p]),
    'sa_vaep_features_conditions': (ctypes.c_int, [ctypes.POINTER(SaActions), ctypes.POINTER(SaFeaturePlan),
                                                   _p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                                   ctypes.c_int32, _p, _p, _p, _p, ctypes.c_int32, _p]),
    'sa_vaep_features_xt': (ctypes.c_int, [ctypes.POINTER(SaActions),
                                           ctypes.POINTER(SaFeaturePlan), ctypes.POINTER(SaBlock),
                                           ctypes.POINTER(SaBlock), ctypes.POINTER(SaBlock),
                                           ctypes.c_int32, ctypes.c_int32, _p, _p]),
    'sa_xt_cells': (ctypes.c_int, [ctypes.POINTER(SaActions), ctypes.c_int32, ctypes.c_int32, _p,
                                   _p]),
    'sa_xt_count_cells': (ctypes.c_int, [_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, _p,
                                         _p, _p, _p, _p, ctypes.c_int32, _p]),
    'sa_xt_rate_cells': (ctypes.c_int, [_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, _p,
                                        _p, _p, _p]),
    'sa_xt_solve': (ctypes.c_int, [_p, _p, _p, _p, ctypes.c_int32, ctypes.c_int32,
                                   ctypes.c_double, ctypes.c_int32, _p, _p, _p,
                                   ctypes.POINTER(ctypes.c_int32), _p]),
    'sa_xt_solve_ex': (ctypes.c_int, [_p, _p, _p, _p, ctypes.c_int32, ctypes.c_int32,
                                      ctypes.c_double, ctypes.c_int32, ctypes.c_int32, _p, _p, _p,
                                      ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32),
                                      _p, _p, _p]),
    'sa_xt_solve_compact': (ctypes.c_int, [_p, _p, _p, _p, _p, _p, ctypes.c_int32, ctypes.c_double,
                                           ctypes.c_int32, ctypes.c_int32, _p,
                                           ctypes.POINTER(ctypes.c_int32),
                                           ctypes.POINTER(ctypes.c_int32), _p]),
    'sa_xt_solve_async': (ctypes.c_int, [_p, _p, _p, _p, ctypes.c_int32, ctypes.c_int32,
                                   ctypes.c_double, ctypes.c_int32, _p, _p, _p,
                                   _p, _p]),
    'sa_xt_normalize': (ctypes.c_int, [_p, _p, _p, _p, ctypes.c_int32, ctypes.c_int32, _p, _p,
                                       _p]),
    'sa_xt_probabilities': (ctypes.c_int, [_p, _p, _p, ctypes.c_int32, _p, _p, _p, _p]),
    'sa_xt_iterate_rows': (ctypes.c_int, [_p, _p, _p, _p, ctypes.c_int32, ctypes.c_int32,
                                          ctypes.c_int32, _p, ctypes.c_double, _p, _p, _p, _p]),
    'sa_xt_band_shape': (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(ctypes.c_int32),
                                        ctypes.POINTER(ctypes.c_int32)]),
    'sa_xt_count_bucket': (ctypes.c_int, [ctypes.POINTER(SaActions), _p, ctypes.c_int64, ctypes.c_int32,
                                          ctypes.c_int32, _p, _p, _p, _p, _p, ctypes.c_int32,
                                          ctypes.c_int32, _p]),
    'sa_xt_rate_interp_codes': (ctypes.c_int, [_p, ctypes.c_int64, _p, _p, _p, ctypes.c_int32,
                                               ctypes.c_int32, _p, ctypes.c_int32, _p, ctypes.c_int32,
                                               _p, _p, _p]),
    'sa_xt_rate_interp_codes_many': (ctypes.c_int, [ctypes.c_int32, ctypes.POINTER(_p),
                                                    ctypes.POINTER(ctypes.c_int64), _p, _p, _p,
                                                    ctypes.c_int32, ctypes.c_int32, _p, ctypes.c_int32,
                                                    _p, ctypes.c_int32, ctypes.POINTER(_p), _p, _p]),
    'sa_xt_fit_rate_interp_codes': (ctypes.c_int, [_p, _p, _p, _p, ctypes.c_int32, ctypes.c_int32,
                                                   ctypes.c_double, ctypes.c_int32, ctypes.c_int32, _p, _p,
                                                   ctypes.POINTER(ctypes.c_int32),
                                                   ctypes.POINTER(ctypes.c_int32), _p, _p, ctypes.c_int32,
                                                   ctypes.POINTER(_p), ctypes.POINTER(ctypes.c_int64), _p, _p,
                                                   _p, ctypes.c_int32, _p, ctypes.c_int32, ctypes.POINTER(_p),
                                                   _p, _p]),
    'sa_xt_count_from_buckets_ex': (ctypes.c_int, [ctypes.c_int32, ctypes.POINTER(_p), ctypes.POINTER(_p),
                                                   ctypes.c_int32, ctypes.c_int32, _p, _p, _p, _p,
                                                   ctypes.c_int32, _p, _p, _p]),
    'sa_xt_count_from_buckets': (ctypes.c_int, [ctypes.c_int32, ctypes.POINTER(_p), ctypes.POINTER(_p),
                                                ctypes.c_int32, ctypes.c_int32, _p, _p, _p, _p,
                                                ctypes.c_int32, _p]),
    'sa_xt_count_band_rows': (ctypes.c_int, [ctypes.c_int32, ctypes.POINTER(_p), ctypes.POINTER(_p),
                                             ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                             ctypes.c_int32, _p, _p, _p, _p, ctypes.c_int32, _p]),
    'sa_xt_compact_bytes': (ctypes.c_int64, [ctypes.c_int32, ctypes.c_int32]),
    'sa_xt_compact_rows': (ctypes.c_int, [_p, ctypes.c_int32, ctypes.c_int32, _p, _p, _p]),
    'sa_xt_iterate_compact': (ctypes.c_int, [_p, _p, _p, _p, _p, _p, ctypes.c_int32, ctypes.c_int32,
                                             ctypes.c_int32, _p, ctypes.c_double, _p, _p, _p, _p]),
    'sa_xt_interp_grid': (ctypes.c_int, [_p, _p, _p, ctypes.c_int32, ctypes.c_int32, _p,
                                         ctypes.c_int32, _p, ctypes.c_int32, _p, _p]),
    'sa_xt_rate': (ctypes.c_int, [ctypes.POINTER(SaActions), _p, ctypes.c_int32, ctypes.c_int32,
                                  _p, _p, _p]),
    'sa_xt_rate_interp': (ctypes.c_int, [ctypes.POINTER(SaActions), _p, _p, _p, ctypes.c_int32,
                                         ctypes.c_int32, _p, ctypes.c_int32, _p, ctypes.c_int32,
                                         _p, _p, _p]),
    'sa_atomic_scratch_bytes': (ctypes.c_int64, [ctypes.c_int64]),
    'sa_atomic_count': (ctypes.c_int, [ctypes.POINTER(SaSpadlFrame), _p,
                                       ctypes.POINTER(ctypes.c_int64), _p]),
    'sa_atomic_emit': (ctypes.c_int, [ctypes.POINTER(SaSpadlFrame), _p,
                                      ctypes.POINTER(SaAtomicFrame), _p]),
    'sa_dribble_count': (ctypes.c_int, [ctypes.POINTER(SaSpadlFrame), ctypes.c_double,
                                        ctypes.c_double, ctypes.c_double, _p, _p, _p,
                                        ctypes.POINTER(ctypes.c_int64),
                                        ctypes.POINTER(ctypes.c_int64), _p]),
    'sa_atomic_passes_flags': (ctypes.c_int, [ctypes.POINTER(SaSpadlFrame), _p, _p]),
    'sa_atomic_passes_emit': (ctypes.c_int, [ctypes.POINTER(SaSpadlFrame), _p, ctypes.c_int64, _p,
                                             ctypes.POINTER(SaSpadlOut), _p]),
    'sa_atomic_count_after_passes': (ctypes.c_int, [ctypes.POINTER(SaSpadlFrame), _p,
                                                    ctypes.POINTER(ctypes.c_int64), _p]),
    'sa_atomic_emit_after_passes': (ctypes.c_int, [ctypes.POINTER(SaSpadlFrame), _p,
                                                   ctypes.POINTER(SaAtomicFrame), _p]),
    'sa_dribble_emit': (ctypes.c_int, [ctypes.POINTER(SaSpadlFrame), ctypes.c_double,
                                       ctypes.c_double, ctypes.c_double, _p, _p,
                                       ctypes.POINTER(SaSpadlOut), _p]),
    'sa_pack_bits': (ctypes.c_int, [ctypes.POINTER(SaBlock), ctypes.c_int64, _p, ctypes.c_int64,
                                    _p]),
    'sa_segment_offsets': (ctypes.c_int, [_p, ctypes.c_int64, ctypes.c_int64, _p, _p]),
    'sa_tree_predict': (ctypes.c_int, [_p, ctypes.c_int32, _p, _p, ctypes.c_int32, _p, ctypes.c_int32,
                                       ctypes.POINTER(SaBlock), ctypes.POINTER(SaBlock),
                                       ctypes.POINTER(SaBlock), ctypes.c_int64, ctypes.c_double,
                                       ctypes.c_int32, ctypes.c_int32, _p, _p]),
    'sa_tree_staged_lds_bytes': (ctypes.c_int64, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32]),
    'sa_tree_predict_staged': (ctypes.c_int, [ctypes.POINTER(SaTreeModel), _p, ctypes.c_int32, _p, _p,
                                              ctypes.c_int32, _p, _p, ctypes.c_int32,
                                              ctypes.POINTER(SaBlock), _p, ctypes.c_int64,
                                              ctypes.POINTER(SaBlock), ctypes.POINTER(SaBlock),
                                              ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, _p]),
    'sa_device_alloc': (ctypes.c_int, [ctypes.c_int64, ctypes.c_int32, ctypes.POINTER(ctypes.c_void_p)]),
    'sa_device_free': (ctypes.c_int, [_p]),
    'sa_copy2d_async': (ctypes.c_int, [_p, ctypes.c_int64, _p, ctypes.c_int64, ctypes.c_int64,
                                       ctypes.c_int64, _p]),
    'sa_event_create': (ctypes.c_int, [ctypes.c_int32, ctypes.POINTER(ctypes.c_void_p)]),
    'sa_event_destroy': (ctypes.c_int, [_p]),
    'sa_event_record': (ctypes.c_int, [_p, _p]),
    'sa_stream_wait_event': (ctypes.c_int, [_p, _p]),
    'sa_event_synchronize': (ctypes.c_int, [_p]),
    'sa_event_elapsed': (ctypes.c_int, [_p, _p, ctypes.POINTER(ctypes.c_float)]),
    'sa_abi_version': (ctypes.c_int, []),
    'sa_segment_blocks': (ctypes.c_int, [_p, ctypes.c_int64, ctypes.c_int64, _p, _p]),
    'sa_last_error': (ctypes.c_char_p, []),
    'sa_build_id': (ctypes.c_char_p, []),
    'sa_debug_enabled': (ctypes.c_int, []),
    'sa_debug_check': (ctypes.c_int, []),
    'sa_debug_xt_solve_abort': (ctypes.c_int, [ctypes.c_int32]),
    'sa_shutdown': (ctypes.c_int, []),
}
EXPORTED_SYMBOLS = tuple(_SIGNATURES)

_lib: Optional[ctypes.CDLL] = None


class NativeError(RuntimeError):
    """A HIP runtime failure inside libsocceraction_amd."""


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """dlopen the library and declare every signature (no GPU needed)."""
    global _lib
    if _lib is not None and path == LIB_PATH:
        return _lib
    if not os.path.exists(path):
        raise ImportError(
            f'{path} is missing: build the HIP library first '
            '(python -m socceraction_amd.build). socceraction_amd has no CPU fallback.')
    # torch ships its own libamdhip64 (SONAME libamdhip64.so.7, same as /opt/rocm's) and
    # device memory comes from torch's allocator, so the process must hold ONE HIP runtime:
    # load torch first and our NEEDED libamdhip64.so.7 binds to that copy.  dlopen-ing this
    # library first would pull in /opt/rocm's runtime as a second instance, and the kernels
    # would then see no device once torch initialises its own.
    import torch  # noqa: F401
    lib = ctypes.CDLL(path)
    for name, (res, args) in _SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.sa_abi_version() != 3:
        raise ImportError('libsocceraction_amd ABI version mismatch')
    _check_build_id(lib, path)
    if path == LIB_PATH:
        _lib = lib
    return lib


def _check_build_id(lib: ctypes.CDLL, path: str) -> None:
    """The default and debug libraries must come from the sources next to them (the build id is
    a hash of the sources, flags and defines; socceraction_amd/build.py)."""
    from . import build as _build
    expected = {DEFAULT_LIB: (), DEBUG_LIB: _build.DEBUG_DEFINES}
    if os.path.abspath(path) not in expected or not os.path.isdir(_build.CSRC):
        return  # an explicitly chosen variant build
    want = _build.build_id(expected[os.path.abspath(path)])
    got = (lib.sa_build_id() or b'').decode()
    if got != want:
        raise ImportError(f'{path} was built from other sources (build id {got}, sources {want}): '
                          'rebuild with python -m socceraction_amd.build')


def lib() -> ctypes.CDLL:
    return load_library()


def shutdown() -> None:
    """Free the library's cached device scratch (sa_shutdown)."""
    if _lib is not None:
        check(_lib.sa_shutdown())


def check(rc: int) -> None:
    """Map a C-ABI status to the reference's exception types.  With the debug build every call
    is followed by the device bounds-check collection (synchronises the device)."""
    if rc == SA_OK and DEBUG:
        rc = lib().sa_debug_check()
    if rc == SA_OK:
        return
    msg = (lib().sa_last_error() or b'').decode(errors='replace')
    if rc in (SA_EINVAL, SA_EDATA):
        raise ValueError(msg)
    if rc == SA_ENOMEM:
        raise MemoryError(msg)
    raise NativeError(f'libsocceraction_amd error {rc}: {msg}')
