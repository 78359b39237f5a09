# QF consumers with an agent-scope acquire after the wait: CLI batch repro x4, batch tests, 8-stream bench
export TMPDIR=/tmp; out=gpurun_out/r05_acq; mkdir -p $out
timeout -k 10 200 python -u tools/r05cli3.py > $out/cli.txt 2>&1 || { echo cli_failed; exit 1; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_llm_batch_gpu.py tests/test_cli_gpu.py > $out/tests.txt 2>&1 || { echo tests_failed; exit 1; }
timeout -k 10 300 python -u bench.py --preset 3 --utts-per-gpu 8 --no-cpu-baseline --batch 0 > $out/b8.json 2> $out/b8.err || { echo b_failed; exit 1; }
echo done
