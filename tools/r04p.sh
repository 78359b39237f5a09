set -e
# env-only A/B on the final batched engine (2.6B Q8_0, 8 streams): steps per graph, attention kind
out=gpurun_out/r04_p
mkdir -p $out
export TMPDIR=/tmp
for r in 1 2; do
for v in "" "MIO_GRAPH_STEPS=16" "MIO_GRAPH_STEPS=4" "MIO_BT_ATT=0"; do
  echo "[$v] $(env $v timeout -k 10 200 python3 tools/batch_prof.py 8 200 4 2>&1 | tail -1)" >> $out/times.txt
done
done
cat $out/times.txt
