"""Build libsocceraction_amd.so in-tree with hipcc for gfx950.

    python -m socceraction_amd.build [--force]

Flags: ``-O3 --offload-arch=gfx950 -ffp-contract=off``.  ``-ffp-contract=off`` is a
parity requirement: numpy evaluates ``dx**2 + dy**2`` and the xT dot products with a
separately rounded multiply and add, so the kernels must not fuse them into FMAs.
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, 'csrc')
OUT = os.path.join(HERE, '_lib', 'libsocceraction_amd.so')
SOURCES = ['sa_api.hip', 'sa_vaep.hip', 'sa_xt.hip', 'sa_atomic.hip', 'sa_trees.hip', 'sa_store.hip']
HEADERS = ['sa_common.h', 'sa_internal.h', os.path.join('..', '..', 'include', 'socceraction_amd.h')]
FLAGS = ['-O3', '--offload-arch=gfx950', '-ffp-contract=off', '-fPIC', '-shared', '-std=c++17',
         '-Wall']


def hipcc() -> str:
    for c in (os.environ.get('HIPCC'), '/opt/rocm/bin/hipcc', 'hipcc'):
        if c and (os.path.sep not in c or os.path.exists(c)):
            return c
    raise RuntimeError('hipcc not found')


def _stale() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS]
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = True, defines=(), out: str = OUT) -> str:
    """Compile the library; ``defines`` (e.g. ``['SA_NT_STORES=0']``) build A/B variants."""
    if out == OUT and not defines and not force and not _stale():
        return out
    os.makedirs(os.path.dirname(out), exist_ok=True)
    tmp = out + '.tmp'
    cmd = [hipcc()] + FLAGS + [f'-D{d}' for d in defines] + \
        [os.path.join(CSRC, s) for s in SOURCES] + ['-o', tmp]
    if verbose:
        print(' '.join(cmd), flush=True)
    subprocess.run(cmd, check=True, cwd=CSRC)
    os.replace(tmp, out)
    return out


if __name__ == '__main__':
    defs = [a[2:] for a in sys.argv[1:] if a.startswith('-D')]
    variant = [a.split('=', 1)[1] for a in sys.argv[1:] if a.startswith('--variant=')]
    target = OUT if not variant else os.path.join(HERE, '_lib', f'libsocceraction_amd_{variant[0]}.so')
    print(build(force='--force' in sys.argv, defines=defs, out=target))
