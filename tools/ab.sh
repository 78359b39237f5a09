# Same-box A/B runner (one gpurun call): runs CMD once per variant per round, variants
# interleaved, each under its own time limit; the JSON each run prints goes to
# gpurun_out/OUT/NAME_ROUND.json (stderr beside it). A variant is NAME[:ENV=V[,ENV=V...]][@BUILD]:
# BUILD is an in-tree build dir (MIO_BUILD_DIR, e.g. miotts-llama.cpp_amd/build_c128 made by
# `make -C miotts-llama.cpp_amd BUILD=build_c128 EXTRA=-DMIO_ATT_CHUNK=128`), ENV the switches.
#   bash tools/ab.sh OUT ROUNDS "python -u tools/llm_ab.py" base c128@miotts-llama.cpp_amd/build_c128 \
#        wgm2:MIO_WGM=2
# Stops at the first failing run (set -e): a failed GPU step ends the call.
set -e
out=gpurun_out/$1; rounds=$2; cmd=$3; shift 3
mkdir -p "$out"
export TMPDIR=/tmp
for r in $(seq 1 "$rounds"); do
  for spec in "$@"; do
    name=${spec%%[:@]*}
    build=""; envs=""
    case "$spec" in *@*) build=${spec##*@};; esac
    rest=${spec%%@*}
    case "$rest" in *:*) envs=$(echo "${rest#*:}" | tr ',' ' ');; esac
    if [ -n "$build" ]; then envs="$envs MIO_BUILD_DIR=$build"; fi
    echo "[ab] round $r $name ($envs)"
    env $envs timeout -k 10 300 $cmd > "$out/${name}_$r.json" 2> "$out/${name}_$r.err"
  done
done
