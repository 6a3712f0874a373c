#!/bin/bash
# (tools/) retry a gpurun call only while the pool reports no free box / busy slots / infra backoff (nothing charged)
out=$1; shift
for i in $(seq 1 12); do
  timeout 3400 /usr/local/graft/bin/gpurun "$@" > "$out" 2>&1
  if grep -q "status=transient" "$out"; then
    w=$(grep -o "retry in [0-9]*s" "$out" | grep -o "[0-9]*" | head -1); w=${w:-180}
    sleep $((w + 20)); continue
  fi
  break
done
