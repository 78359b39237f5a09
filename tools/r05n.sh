# the attention block in one launch (k_layer_att): parity, timeline, bench A/B
export TMPDIR=/tmp; out=gpurun_out/r05_n; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_llm_layers_gpu.py -x -q --timeout 120 --timeout-method thread > $out/layers.log 2>&1 || { echo layers_failed; exit 1; }
timeout -k 10 200 python -u tools/step_timeline.py > $out/timeline.txt 2>&1 || { echo timeline_failed; exit 1; }
timeout -k 10 500 python -u -m pytest tests/test_llm_gpu.py tests/test_lfm2_gpu.py tests/test_llm_batch_gpu.py -x -q --timeout 200 --timeout-method thread > $out/llm.log 2>&1 || { echo llm_failed; exit 1; }
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-cpu-c1 > $out/fused.json 2> $out/fused.err || { echo bench_failed; exit 1; }
MIO_LAYER_ATT=0 timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-cpu-c1 > $out/att_o.json 2> $out/att_o.err || { echo bench0_failed; exit 1; }
echo done
