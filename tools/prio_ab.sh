#!/bin/bash
# C5 stream benchmark under stream-priority settings (codec stream / device stream), one
# JSON line each: usage bash tools/prio_ab.sh OUT
set -e
out=${1:-gpurun_out/prio}
mkdir -p $out
python3 -c "import ctypes; h=ctypes.CDLL('/opt/rocm/lib/libamdhip64.so'); a=ctypes.c_int(); b=ctypes.c_int(); h.hipDeviceGetStreamPriorityRange(ctypes.byref(a), ctypes.byref(b)); print('priority range least', a.value, 'greatest', b.value)" > $out/range.txt
for cfg in "normal normal" "low normal" "normal high" "low high" "normal normal"; do
  set -- $cfg
  echo "{\"cstream\": \"$1\", \"stream\": \"$2\"}" >> $out/ab.jsonl
  MIO_CSTREAM_PRIO=$1 MIO_STREAM_PRIO=$2 AB_K=3 timeout -k 10 300 python3 tools/stream_ab.py >> $out/ab.jsonl
done
