#!/bin/bash
# same-box A/B of the steps per replayed step graph (MIO_GRAPH_STEPS), poll cadence 32
set -e
out=${1:-gpurun_out/gsteps}
mkdir -p $out
for v in 8 32 16 8 32 16; do
  echo "{\"MIO_GRAPH_STEPS\": $v}" >> $out/ab.jsonl
  MIO_GRAPH_STEPS=$v AB_CI=32 AB_K=4 timeout -k 10 200 python3 tools/llm_ab.py >> $out/ab.jsonl
done
