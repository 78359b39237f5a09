# Same-box A/B of several builds, alternating: ab_multi.sh ROUNDS NAME:DIR [NAME:DIR ...]
# bench JSON of each run -> gpurun_out/abm_NAME_ROUND.json
set -e
rounds=$1; shift
for r in $(seq 1 $rounds); do
  for pair in "$@"; do
    name=${pair%%:*}; dir=${pair#*:}
    MIO_BUILD_DIR=$dir timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --batch 0 > gpurun_out/abm_${name}_$r.json 2> gpurun_out/abm_${name}_$r.err
  done
done
