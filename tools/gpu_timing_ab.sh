cd ${GRAFT_REPO_ROOT:-$(pwd)}
for r in 1 2 3; do
  for t in on off; do
    if [ $t = off ]; then X=--no-kernel-timing; else X=; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --channels 2048 $X > gpurun_out/tim_${t}_$r.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/tim_${t}_$r.json'));print('$t', $r, d['ms_per_step'])"
  done
done
