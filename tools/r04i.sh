set -e
# eager kernel stats of the 8-stream 2.6B Q8_0 step with MIO_BT_FQ=1 (default) and 3
out=gpurun_out/r04_i
mkdir -p $out
export TMPDIR=/tmp MIO_NO_GRAPH=1
for fqv in 1 3; do
MIO_BT_FQ=$fqv timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/k$fqv -o k -- python3 tools/batch_prof.py 8 48 4 > $out/k$fqv.out 2>&1
done
echo done
