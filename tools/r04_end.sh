set -e
# final code of the session: every GPU test, the default bench line, C4, smoke
out=gpurun_out/r04_end
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1
timeout -k 10 400 python -u bench.py > $out/bench.json 2> $out/bench.err
timeout -k 10 400 python -u bench.py --preset 4 --utts-per-gpu 8 --steps 2 --warmup 1 --no-cpu-baseline > $out/c4_bench.json 2> $out/c4_bench.err
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1
tail -1 $out/gpu_tests.log
