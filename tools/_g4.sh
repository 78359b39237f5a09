set -e
out=gpurun_out/r04_full1
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -3 $out/tests.log
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 > $out/bench.json 2> $out/bench.err
cat $out/bench.json
