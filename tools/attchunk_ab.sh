#!/bin/bash
# same-box A/B of the decode attention chunk (kAttChunk 128 = build, 64 = build_c64)
set -e
out=${1:-gpurun_out/attchunk}
mkdir -p $out
for b in ${AB_BUILDS:-build build_c64 build build_c64}; do
  MIO_BUILD_DIR=miotts-llama.cpp_amd/$b AB_CI=32 AB_K=4 timeout -k 10 200 python3 tools/llm_ab.py >> $out/ab.jsonl
done
