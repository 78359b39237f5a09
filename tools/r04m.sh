set -e
# engine-choice A/B on the current batched engine, then the round-end pass
out=gpurun_out/r04_m
mkdir -p $out
export TMPDIR=/tmp
for v in "" "MIO_MMQ_MASK=0" "MIO_BT_FQ=3" "MIO_MMQ_MASK=0 MIO_BT_FQ=3"; do
  for p in 3 4; do
    echo "[$v] p$p $(env $v timeout -k 10 200 python3 tools/batch_prof.py 8 200 $p 2>&1 | tail -1)" >> $out/times.txt
  done
done
cat $out/times.txt
bash tools/r04_final.sh
