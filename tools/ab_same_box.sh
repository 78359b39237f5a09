# Same-box A/B of two builds, alternating runs (bench + timeline each): ab_same_box.sh NAME_A DIR_A NAME_B DIR_B [rounds]
set -e
rounds=${5:-2}
for r in $(seq 1 $rounds); do
  for pair in "$1:$2" "$3:$4"; do
    name=${pair%%:*}; dir=${pair#*:}
    MIO_BUILD_DIR=$dir timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab_${name}_$r.json 2> gpurun_out/ab_${name}_$r.err
  done
done
