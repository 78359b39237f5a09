set -e
# C5 streaming: codec GEMM K-groups (LDS footprint per block) and codec stream priority vs
# the LLM steps it overlaps
out=gpurun_out/r03_n
mkdir -p $out
export TMPDIR=/tmp
AB_K=3 timeout -k 10 200 python -u tools/stream_ab.py > $out/c5_default.jsonl 2>&1
MIO_CODEC_KG=1 AB_K=3 timeout -k 10 200 python -u tools/stream_ab.py > $out/c5_kg1.jsonl 2>&1
MIO_CODEC_KG=2 AB_K=3 timeout -k 10 200 python -u tools/stream_ab.py > $out/c5_kg2.jsonl 2>&1
MIO_CSTREAM_PRIO=low AB_K=3 timeout -k 10 200 python -u tools/stream_ab.py > $out/c5_low.jsonl 2>&1
AB_K=3 timeout -k 10 200 python -u tools/stream_ab.py > $out/c5_default2.jsonl 2>&1
