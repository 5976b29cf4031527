#!/bin/bash
# Runs one GPU step under a time limit; exit status 0/1 (pass / test failure) lets the caller
# continue, anything else (timeout 124/137, abort 134, segfault 139, ...) ends the call.
# usage: tools/gpu_step.sh SECONDS LOG cmd...
t=$1; log=$2; shift 2
timeout -k 10 "$t" "$@" >> "$log" 2>&1
rc=$?
echo "[gpu_step] rc=$rc: $*" >> "$log"
if [ $rc -gt 1 ]; then echo "[gpu_step] stopping after rc=$rc" >> "$log"; exit $rc; fi
exit 0
