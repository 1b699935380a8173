#!/bin/bash
# Host-side helper (not run on the GPU box): run one gpurun call, and again only while the pool reports
# that nothing ran (no box / slot free, or access backing off).  usage: gpurun_retry.sh OUTFILE TIMEOUT CMD
out=$1; to=$2; shift 2
for i in $(seq 1 15); do
  /usr/local/graft/bin/gpurun --timeout $to -- "$@" > $out 2>&1
  if grep -qE "no free box|slot\(s\) on this pod are busy|backing off" $out; then sleep 360; continue; fi
  break
done
