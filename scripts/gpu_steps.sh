#!/bin/bash
# step NAME SECONDS CMD...: one GPU step under its own time limit, output in
# $O/NAME.log, "NAME rc=N" appended to $O/steps.log; returns the step's rc.
step() {
  local name=$1 t=$2
  shift 2
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a "$O/steps.log"
  return $rc
}
