# One GPU-box pass: GPU tests, the default bench line (with the CPU baseline), the eager
# bench under rocprofv3 kernel trace + stats (graph replays crash rocprofiler-sdk 7.2's
# queue intercept), and the two PMC passes at decode position ~400.
# With "configs" as the third argument, also smoke() and the BASELINE config lines C2 (0.1B
# Q8_0), C4 (2.6B Q8_0, 8 utterances per GPU; the plain-attention stand-in and the LFM2-2.6B shape)
# and C5 (stream benchmark, 3 runs).
# Outputs under gpurun_out/$TAG/.   usage: bash tools/gpu_round.sh TAG [skip-tests|tests] [configs]
set -e
tag=${1:-run}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1
fi
timeout -k 10 400 python -u bench.py > $out/bench.json 2> $out/bench.err
MIO_NO_GRAPH=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --batch 0 > $out/bench_prof.json 2> $out/prof.err
find $out/prof -name '*kernel_stats.csv' -exec cp {} $out/kernel_stats.csv \;
rm -rf $out/prof  # the full trace exceeds gpurun's 64 MiB copy-back
MIO_NO_GRAPH=1 timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $out/pmc -o fetch -- python3 tools/pmc_run.py > $out/pmc_fetch.out 2>&1
MIO_NO_GRAPH=1 timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $out/pmc -o write -- python3 tools/pmc_run.py > $out/pmc_write.out 2>&1
python3 tools/pmc_traffic.py $(find $out/pmc -name 'fetch_counter_collection.csv') $(find $out/pmc -name 'write_counter_collection.csv') 3 > $out/pmc_traffic.json
find $out/pmc -name '*kernel_trace.csv' -delete
if [ "$3" = "configs" ]; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.txt 2>&1
  timeout -k 10 400 python -u bench.py --preset 2 --no-cpu-baseline > $out/c2.json 2> $out/c2.err
  timeout -k 10 400 python -u bench.py --preset 4 --utts-per-gpu 8 --no-cpu-baseline --batch 0 > $out/c4.json 2> $out/c4.err
  timeout -k 10 400 python -u bench.py --preset 6 --utts-per-gpu 8 --no-cpu-baseline --batch 0 > $out/c4_lfm2.json 2> $out/c4_lfm2.err
  AB_K=3 timeout -k 10 400 python -u tools/stream_ab.py > $out/c5.json 2> $out/c5.err
fi
echo done
