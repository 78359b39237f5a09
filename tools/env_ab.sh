set -e
for spec in base "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1" "ROC_SYSTEM_SCOPE_SIGNAL=0" "AMD_DIRECT_DISPATCH=0" "DEBUG_CLR_KERNARG_HDP_FLUSH_WA=0"; do
  if [ "$spec" = base ]; then envs=""; else envs="$spec"; fi
  env $envs timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/env_$(echo $spec | tr '=' '_').json 2>/dev/null || echo "fail $spec"
done
