set -e
# the BASELINE configuration lines on the current code (one box): C3 + batched, C2, C4 per GPU,
# C5 streaming; then smoke
out=gpurun_out/${OUT:-r04_cfg}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > $out/c3_bench.json 2> $out/c3_bench.err
timeout -k 10 300 python -u bench.py --preset 2 --steps 5 --warmup 1 --no-cpu-baseline --batch 0 > $out/c2_bench.json 2> $out/c2_bench.err
timeout -k 10 400 python -u bench.py --preset 4 --utts-per-gpu 8 --steps 2 --warmup 1 --no-cpu-baseline > $out/c4_bench.json 2> $out/c4_bench.err
AB_K=3 timeout -k 10 300 python -u tools/stream_ab.py > $out/c5_stream.jsonl 2> $out/c5_stream.err
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1
