"""Build libsocceraction_amd.so in-tree with hipcc for gfx950.

    python -m socceraction_amd.build [--force] [--debug] [-DNAME=V ... --variant=tag]

Flags: ``-O3 --offload-arch=gfx950 -ffp-contract=off``.  ``-ffp-contract=off`` is a
parity requirement: numpy evaluates ``dx**2 + dy**2`` and the xT dot products with a
separately rounded multiply and add, so the kernels must not fuse them into FMAs.

Every build embeds a build id -- a hash of the sources, headers, flags and defines -- as
``sa_build_id()`` and as a ``sa-build-id:<hash>`` marker in the file.  A library is rebuilt
when its marker differs from the hash of the current sources (not by file times), and
``_native.load_library()`` refuses a library whose id does not match the sources next to it.
``--debug`` builds ``libsocceraction_amd_debug.so`` with the device bounds checks of
``csrc/sa_debug.h`` (``-DSA_DEBUG=1``).
"""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys
from typing import Sequence

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, 'csrc')
LIBDIR = os.path.join(HERE, '_lib')
OUT = os.path.join(LIBDIR, 'libsocceraction_amd.so')
DEBUG_OUT = os.path.join(LIBDIR, 'libsocceraction_amd_debug.so')
SOURCES = ['sa_api.hip', 'sa_vaep.hip', 'sa_xt.hip', 'sa_xt_large.hip', 'sa_atomic.hip', 'sa_trees.hip', 'sa_store.hip']
HEADERS = ['sa_common.h', 'sa_internal.h', 'sa_debug.h',
           os.path.join('..', '..', 'include', 'socceraction_amd.h')]
FLAGS = ['-O3', '--offload-arch=gfx950', '-ffp-contract=off', '-fPIC', '-shared', '-std=c++17',
         '-Wall']
DEBUG_DEFINES = ('SA_DEBUG=1',)


def hipcc() -> str:
    for c in (os.environ.get('HIPCC'), '/opt/rocm/bin/hipcc', 'hipcc'):
        if c and (os.path.sep not in c or os.path.exists(c)):
            return c
    raise RuntimeError('hipcc not found')


def build_id(defines: Sequence[str] = ()) -> str:
    """Hash of every source and header, the flags and the defines (16 hex digits)."""
    h = hashlib.sha256()
    for f in SOURCES + HEADERS:
        with open(os.path.join(CSRC, f), 'rb') as fh:
            h.update(f.encode() + b'\0' + fh.read() + b'\0')
    h.update(' '.join(FLAGS + sorted(defines)).encode())
    return h.hexdigest()[:16]


def file_build_id(path: str):
    """The build id marker of a built library file, or None."""
    try:
        with open(path, 'rb') as fh:
            data = fh.read()
    except OSError:
        return None
    i = data.find(b'sa-build-id:')
    if i < 0:
        return None
    return data[i + 12:i + 28].decode(errors='replace')


def build(force: bool = False, verbose: bool = True, defines: Sequence[str] = (), out: str = OUT) -> str:
    """Compile the library; ``defines`` (e.g. ``['SA_NT_STORES=0']``) build A/B variants."""
    bid = build_id(defines)
    if not force and file_build_id(out) == bid:
        return out
    os.makedirs(os.path.dirname(out), exist_ok=True)
    tmp = out + '.tmp'
    cmd = [hipcc()] + FLAGS + [f'-D{d}' for d in defines] + [f'-DSA_BUILD_ID="{bid}"'] + \
        [os.path.join(CSRC, s) for s in SOURCES] + ['-o', tmp]
    if verbose:
        print(' '.join(cmd), flush=True)
    subprocess.run(cmd, check=True, cwd=CSRC)
    os.replace(tmp, out)
    return out


def build_debug(force: bool = False, verbose: bool = True) -> str:
    return build(force=force, verbose=verbose, defines=DEBUG_DEFINES, out=DEBUG_OUT)


if __name__ == '__main__':
    defs = [a[2:] for a in sys.argv[1:] if a.startswith('-D')]
    variant = [a.split('=', 1)[1] for a in sys.argv[1:] if a.startswith('--variant=')]
    if '--debug' in sys.argv:
        print(build_debug(force='--force' in sys.argv))
    else:
        target = OUT if not variant else os.path.join(LIBDIR, f'libsocceraction_amd_{variant[0]}.so')
        print(build(force='--force' in sys.argv, defines=defs, out=target))
