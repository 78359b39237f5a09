export TMPDIR=/tmp; out=gpurun_out/r05_cl; mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_cli_gpu.py > $out/tests.txt 2>&1 || { echo tests_failed; exit 1; }
echo done
