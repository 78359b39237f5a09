# One GPU-box pass: GPU tests, the default bench line (with the CPU baseline), then the
# graph-mode bench under rocprofv3 kernel trace + stats. Outputs under gpurun_out/$TAG/.
# usage: bash tools/gpu_round.sh TAG [skip-tests]
set -e
tag=${1:-run}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1
fi
timeout -k 10 400 python -u bench.py > $out/bench.json 2> $out/bench.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --batch 0 > $out/bench_prof.json 2> $out/prof.err
find $out/prof -name '*kernel_stats.csv' -exec cp {} $out/kernel_stats.csv \;
rm -rf $out/prof  # the full trace exceeds gpurun's 64 MiB copy-back
echo done
