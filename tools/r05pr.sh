# layer_att policy: fusion bit-identity (forced on preset 2), layers, lfm2 kinds, C2 bench with the policy
export TMPDIR=/tmp; out=gpurun_out/r05_pr; mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_llm_gpu.py tests/test_lfm2_gpu.py > $out/tests.txt 2>&1 || { echo tests_failed; exit 1; }
timeout -k 10 300 python -u bench.py --preset 2 --no-cpu-baseline --no-cpu-c1 --batch 0 > $out/c2.json 2> $out/c2.err || { echo b_failed; exit 1; }
echo done
