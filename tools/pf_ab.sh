#!/bin/bash
# same-box A/B of two builds on the LLM-only bench workload (68-token prompt + 700 tokens)
set -e
out=${1:-gpurun_out/pfab}
mkdir -p $out
for r in 1 2 3; do
  for b in build_a build; do
    echo "{\"build\": \"$b\"}" >> $out/ab.jsonl
    MIO_BUILD_DIR=miotts-llama.cpp_amd/$b AB_CI=32 timeout -k 10 200 python3 tools/llm_ab.py >> $out/ab.jsonl
  done
done
