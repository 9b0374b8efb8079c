"""socceraction_amd — MI355X-native valuation path of socceraction.

Drop-in module layout (``socceraction_amd.vaep``, ``.atomic.vaep``, ``.xthreat``,
``.spadl``) over hand-written HIP kernels for gfx950 reached through the C ABI in
``include/socceraction_amd.h``. Importing the package needs no GPU; computing does.
"""
__version__ = '0.1.0'
