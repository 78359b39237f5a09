# Same-box A/B of the fused attention (MIO_ATT_FUSED=1, default) against attention as its own
# launch (0): LLM GPU tests first, then interleaved bench lines.  usage: bash tools/att_ab.sh TAG [tests]
set -e
tag=${1:-att}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
if [ "$2" = "tests" ]; then
  MIO_ATT_FUSED=1 timeout -k 10 600 python -u -m pytest tests/test_llm_gpu.py tests/test_cli_gpu.py -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1
fi
for r in 1 2; do
  for f in 0 1; do
    MIO_ATT_FUSED=$f timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --batch 0 > $out/bench_f${f}_r$r.json 2> $out/bench_f${f}_r$r.err
    echo "fused=$f run=$r $(python3 -c "import json,sys; d=json.load(open('$out/bench_f${f}_r$r.json')); print(d['value'], d['llm_ms_per_token'], d['roofline']['per_token_us'])")"
  done
done
