# round-4: VQ kernel templated on D -- same-box A/B against the previous commit's tree (ab_head/)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4u; mkdir -p $O
for pass in 0 1; do
  for t in new old; do
    d=$([ $t = new ] && echo . || echo ab_head)
    (cd $d && timeout -k 10 300 python bench.py --no-cpu-baseline --fp32-steps 0 --steps 40 --vq-reps 200) > $O/b_${t}_$pass.json 2> $O/b_${t}_$pass.err || exit $?
    python3 -c "
import json; d=json.load(open('$O/b_${t}_$pass.json')); print('$t', $pass, d['value'], d['ms_per_step'], d['vq']['us'], d['vq']['us_with_stats'])"
  done
done
