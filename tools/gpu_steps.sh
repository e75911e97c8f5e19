#!/bin/bash
# GPU job helper: `source tools/gpu_steps.sh`, then `step SECONDS 'command'`
# per GPU step.  Each step runs under its own time limit; an ordinary failure
# (exit 1: a failed test, a Python exception) lets the next step run, while a
# fault, abort, segfault, time limit or any other status ends the job there
# (no further GPU work in a call after trouble).
STEP_RC=0
step() {
  local t=$1
  shift
  echo "[step] $* (limit ${t}s)"
  timeout -k 10 "$t" bash -c "$*"
  local rc=$?
  echo "[step] rc=$rc"
  [ $rc -ne 0 ] && STEP_RC=$rc
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "[step] stopping: status $rc"
    exit $rc
  fi
  return 0
}
