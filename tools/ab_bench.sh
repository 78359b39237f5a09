# A/B bench runs on the GPU box: each argument is NAME or NAME:VAR=VAL[,VAR=VAL...]; the bench
# JSON of each goes to gpurun_out/ab_NAME.json (and the step timeline to ab_NAME.tl.txt).
set -e
for spec in "$@"; do
  name=${spec%%:*}
  envs=""
  if [ "$spec" != "$name" ]; then envs=$(echo "${spec#*:}" | tr ',' ' '); fi
  env $envs timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err
  env $envs timeout -k 10 300 python tools/step_timeline.py --pos 400 > gpurun_out/ab_$name.tl.txt 2>/dev/null
done
