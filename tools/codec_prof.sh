#!/bin/bash
# usage: tools/codec_prof.sh OUTDIR TAG [ENV=VAL ...] -- eager kernel trace of the T=700 codec
# decode (second of two runs) -> OUTDIR/TAG.report.txt
set -e
out=$1; tag=$2; shift 2
mkdir -p "$out"
export TMPDIR=/tmp
env "$@" timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d /tmp/ct_$tag -o run -- python3 tools/codec_trace.py > "$out/$tag.run.txt" 2>&1
python3 tools/codec_trace.py --report $(find /tmp/ct_$tag -name "*kernel_trace.csv") > "$out/$tag.report.txt"
grep -a "codec ms" "$out/$tag.run.txt"
