#!/bin/bash
# A/B of runtime switches: each argument is "tag:VAR=V[,VAR=V...]" (tag only = defaults).
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; mkdir -p gpurun_out
for spec in "$@"; do
  tag=${spec%%:*}; vars=""
  [[ "$spec" == *:* ]] && vars=${spec#*:}
  envs=(); IFS=',' read -ra kv <<< "$vars"; for x in "${kv[@]}"; do [ -n "$x" ] && envs+=("$x"); done
  env "${envs[@]}" timeout -k 10 120 python bench.py --no-cpu-baseline --steps ${AB_STEPS:-100} > gpurun_out/ab_$tag.json 2> gpurun_out/ab_$tag.err || { tail -5 gpurun_out/ab_$tag.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ab_$tag.json'));print('$tag', d['value'], d['ms_per_step'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"
done
