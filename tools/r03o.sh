set -e
# single-launch GroupNorm: codec parity suite, codec time, C5 streaming (sliced path A/B)
out=gpurun_out/r03_o
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_codec_gpu.py tests/test_cli_gpu.py > $out/tests.log 2>&1
timeout -k 10 200 python3 tools/codec_time.py > $out/codec_time.txt 2>&1
MIO_GN_SLICED=1 timeout -k 10 200 python3 tools/codec_time.py > $out/codec_time_sliced.txt 2>&1
AB_K=3 timeout -k 10 200 python -u tools/stream_ab.py > $out/c5.jsonl 2>&1
MIO_GN_SLICED=1 AB_K=3 timeout -k 10 200 python -u tools/stream_ab.py > $out/c5_sliced.jsonl 2>&1
AB_K=3 timeout -k 10 200 python -u tools/stream_ab.py > $out/c5_b.jsonl 2>&1
