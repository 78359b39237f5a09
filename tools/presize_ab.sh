#!/bin/bash
# C5 stream benchmark with the PCM buffer pre-sized (default) vs grown per re-decode
set -e
out=${1:-gpurun_out/presize}
mkdir -p $out
for v in 1 0 1 0; do
  echo "{\"MIO_STREAM_PRESIZE\": $v}" >> $out/ab.jsonl
  MIO_STREAM_PRESIZE=$v AB_K=3 timeout -k 10 300 python3 tools/stream_ab.py >> $out/ab.jsonl
done
