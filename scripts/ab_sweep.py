"""A/B sweep of library variants: runs bench.py once per (round, variant), interleaved.

    python scripts/ab_sweep.py ROUNDS variant1 variant2 ...   ('default' = the main library)

A variant may carry bench arguments after '@', e.g. 'default@--tile-rows=0' (plain layout).

Each run is a fresh process with SOCCERACTION_AMD_LIB pointing at
socceraction_amd/_lib/libsocceraction_amd_<variant>.so; results go to gpurun_out/ab.json.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    rounds = int(sys.argv[1])
    variants = sys.argv[2:]
    res = {v: [] for v in variants}
    for r in range(rounds):
        for spec in variants:
            v, _, extra = spec.partition('@')
            env = dict(os.environ)
            if v != 'default':
                env['SOCCERACTION_AMD_LIB'] = os.path.join(
                    ROOT, 'socceraction_amd', '_lib', f'libsocceraction_amd_{v}.so')
            args = [sys.executable, 'bench.py', '--steps', '20', '--warmup', '3', '--no-cpu']
            args += [a for a in extra.split(',') if a]
            out = subprocess.run(args, cwd=ROOT, env=env, capture_output=True, text=True,
                                 timeout=300)
            line = [ln for ln in out.stdout.splitlines() if ln.startswith('{')]
            if out.returncode != 0 or not line:
                print(spec, 'FAILED', out.returncode, out.stderr[-2000:], flush=True)
                sys.exit(out.returncode or 1)
            d = json.loads(line[0])
            ks = {k: x['ms'] for k, x in d['kernels'].items()}
            res[spec].append({'ms_per_step': d['ms_per_step'], 'kernels': ks})
            print(r, spec, d['ms_per_step'], ks, flush=True)
    os.makedirs(os.path.join(ROOT, 'gpurun_out'), exist_ok=True)
    with open(os.path.join(ROOT, 'gpurun_out', 'ab.json'), 'w') as f:
        json.dump(res, f, indent=1)


if __name__ == '__main__':
    main()
