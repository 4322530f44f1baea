#!/bin/bash
# Run GPU steps in order; each under its own time limit; stop at the first failing step
# (a GPU fault surfaces as an ordinary Python error too), so nothing else touches a sick GPU.
# usage: scripts/gpu_session.sh "name:seconds:command" ...
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
  echo "== $name ($secs s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc"; tail -4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "step failed ($rc): stopping"; exit $rc; fi
done
