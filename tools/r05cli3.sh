export TMPDIR=/tmp; out=gpurun_out/r05_cli3; mkdir -p $out
timeout -k 10 500 python -u tools/r05cli3.py > $out/cli.txt 2>&1 || { echo cli_failed; exit 1; }
echo done
