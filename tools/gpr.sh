#!/bin/bash
# local helper (this container): run a gpurun call, retrying only while gpurun reports no free box (exit 3: nothing ran)
# usage: gpr.sh <logfile> <timeout> <command>   -- retries only while gpurun reports no free box (exit 3)
log=$1; to=$2; shift 2
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout $to -- "$@" > $log 2>&1; rc=$?
  echo "EXIT $rc" >> $log
  [ $rc -ne 3 ] && exit $rc
  sleep 150
done
