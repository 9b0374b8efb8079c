"""The compact xT iteration's quotient (xt_iter_ell_kernel, SA_XE_QDIV): cnt / move formed as a
reciprocal product plus one fma correction must be the IEEE quotient bit for bit (the reference
divides, xthreat.py:_get_transition_matrix); so must the binning's x / 105 and y / 68 (bin_quot,
sa_common.h; xthreat.py:_get_cell_indexes).  scripts/check_quotient.c checks the identity on
the host in double arithmetic -- the same operations the kernel issues (v_rcp-free division for
the reciprocal, v_mul_f64, two v_fma_f64).  A reduced sweep here; the full one (every count
< 65536 x 12001 divisors + 4e8 random pairs) is the program's default."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which('gcc') is None, reason='needs gcc')
def test_fma_corrected_quotient_is_the_ieee_quotient(tmp_path):
    exe = tmp_path / 'check_quotient'
    subprocess.run(['gcc', '-O2', '-ffp-contract=off', os.path.join(ROOT, 'scripts', 'check_quotient.c'),
                    '-o', str(exe), '-lm'], check=True)
    r = subprocess.run([str(exe), '300', '3000000'], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip().endswith('bad=0'), r.stdout
