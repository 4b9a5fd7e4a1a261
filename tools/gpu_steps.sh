#!/bin/bash
# Run GPU steps in order, each under its own time limit, output to gpurun_out/<dir>/<name>.log.
# A step that fails normally (exit 1: a failed test / assertion) does not stop the chain; any other
# status (fault, abort 134, segfault 139, time limit 124/137) ends the call there.
# usage: tools/gpu_steps.sh <outdir> "name|seconds|command" ...
out=$1; shift
mkdir -p "$out"
for step in "$@"; do
    name=${step%%|*}; rest=${step#*|}; secs=${rest%%|*}; cmd=${rest#*|}
    echo "== $name ($secs s): $cmd"
    timeout -k 10 "$secs" bash -c "$cmd" > "$out/$name.log" 2>&1
    rc=$?
    echo "== $name rc=$rc"; tail -n 4 "$out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
done
