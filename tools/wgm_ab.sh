#!/bin/bash
# same-box A/B of matvec workgroups per CU (MIO_WGM) with the lm_head kept at 2 per CU
set -e
out=${1:-gpurun_out/wgm}
mkdir -p $out
for v in "1 2" "2 1" "1 2" "2 1"; do
  set -- $v
  echo "{\"MIO_WGM\": $1, \"MIO_LM_WGM\": $2}" >> $out/ab.jsonl
  MIO_WGM=$1 MIO_LM_WGM=$2 AB_CI=32 timeout -k 10 200 python3 tools/llm_ab.py >> $out/ab.jsonl
done
