# One GPU-box pass: GPU tests, the default bench line (with the CPU baseline), then the
# same bench under rocprofv3 kernel trace + stats. Outputs under gpurun_out/$TAG/.
# usage: bash tools/gpu_round.sh TAG [skip-tests]
set -e
tag=${1:-run}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1
fi
timeout -k 10 400 python -u bench.py > $out/bench.json 2> $out/bench.err
# graph replays crash rocprofv3's kernel tracer on this ROCm: profile the eager launches
# (same kernels, same arguments; MIO_NO_GRAPH=1, csrc/host/llm.cpp llm_run)
MIO_NO_GRAPH=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $out/bench_prof.json 2> $out/prof.err
find $out/prof -name '*kernel_stats.csv' -exec cp {} $out/kernel_stats.csv \;
rm -rf $out/prof  # the full trace exceeds gpurun's 64 MiB copy-back
echo done
