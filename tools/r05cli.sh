export TMPDIR=/tmp; out=gpurun_out/r05_cli; mkdir -p $out
timeout -k 10 600 python -u tools/r05cli.py > $out/cli.txt 2>&1 || { echo cli_failed; exit 1; }
echo done
