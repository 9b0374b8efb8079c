#!/usr/bin/env bash
# rocprofv3 passes for the bench: kernel trace + stats, then one PMC pass per TCC counter group
# (FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950). Outputs under gpurun_out/.
# The trace and PMC passes run the step alone (--no-side: every launch of a step kernel has
# the step's size, so the averages are the step's); the "side" trace adds the side entries.
set -euo pipefail
export TMPDIR=/tmp
tag=${1:-r01}
steps=${2:-10}
mkdir -p gpurun_out
# the build the counters are taken on (bench.py quotes roofline.traffic only for this build)
python3 -c "import sys; sys.path.insert(0, '.'); from socceraction_amd.build import file_build_id, OUT; print(file_build_id(OUT))" \
  > gpurun_out/prof_${tag}_build_id.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag}_trace -o run \
  -- python3 bench.py --steps "$steps" --warmup 2 --no-cpu --no-side > gpurun_out/prof_${tag}_trace.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag}_side -o run \
  -- python3 bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/prof_${tag}_side.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_${tag}_fetch -o run \
  -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-side > gpurun_out/prof_${tag}_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_${tag}_write -o run \
  -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-side > gpurun_out/prof_${tag}_write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/prof_${tag}_hit -o run \
  -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-side > gpurun_out/prof_${tag}_hit.log 2>&1 || echo "hit pass failed"
echo profile done
