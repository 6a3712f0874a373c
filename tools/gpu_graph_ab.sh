#!/bin/bash
# Round-5 A/B: what do HIP graphs buy the pipelined bench, with and without the runtime's graph packet
# capture?  (a) graphs on (default runtime), (b) graphs off (direct launches), (c) graphs on with
# DEBUG_CLR_GRAPH_PACKET_CAPTURE=0; alternated twice.  Headline pass only.
mkdir -p gpurun_out
B="python -u bench.py --no-extras --no-cpu-baseline --steps 20 --warmup 5"
for r in 1 2; do
  for v in a b c; do
    case $v in
      a) E="";;
      b) E="PITT_GRAPHS=0";;
      c) E="DEBUG_CLR_GRAPH_PACKET_CAPTURE=0";;
    esac
    env $E timeout -k 10 300 $B > gpurun_out/gab_${v}${r}.json 2> gpurun_out/gab_${v}${r}.log || { echo "$v$r failed"; tail -5 gpurun_out/gab_${v}${r}.log; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/gab_${v}${r}.json')); print('$v$r', d['value'], d['ms_per_step'], d['hip_graphs'])"
  done
done
