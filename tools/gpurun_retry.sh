#!/bin/bash
# Local helper (runs in the build container, not on the GPU box): one gpurun call; when the infrastructure gave no box
# (status transient / no slot, nothing ran), wait and ask again; never retries a command that ran
out=$1; shift
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun "$@" > "$out" 2>&1
  rc=$?
  if grep -q "status=transient\|no free box\|slot(s) on this pod are busy\|backing off" "$out" && ! grep -q "status=ok" "$out"; then
    echo "attempt $i: transient (rc=$rc), retrying in 60s" >> "$out.attempts"; sleep 60; continue
  fi
  break
done
