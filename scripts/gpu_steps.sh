#!/usr/bin/env bash
# Run GPU steps in order, each under its own time limit, logging to gpurun_out/.
# Continues past ordinary failures (exit 1/2: failed tests / python errors) but stops at
# the first fault-like status (abort 134, segfault 139, timeout 124/137, or signals).
# usage: scripts/gpu_steps.sh NAME:SECONDS:'command' ...
set -u
mkdir -p gpurun_out
rc_all=0
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== [$name] ($secs s) $cmd" | tee -a gpurun_out/steps.log
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc after $(( $(date +%s) - start )) s" | tee -a gpurun_out/steps.log
  tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then rc_all=$rc; fi
  case $rc in
    0|1|2|4|5) ;;
    *) echo "=== stopping: fault-like exit status $rc" | tee -a gpurun_out/steps.log; exit $rc ;;
  esac
done
exit $rc_all
