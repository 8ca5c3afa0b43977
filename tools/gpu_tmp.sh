set -e
cd $GRAFT_REPO_ROOT
for v in "4 4" "8 2" "8 4"; do
  set -- $v
  SKY_DOM_PPT=$1 SKY_DOM_R=$2 timeout -k 10 120 python bench.py --tuples 10000000 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ab_$1_$2.json 2>/dev/null
  python -c "import json,sys; d=json.loads(open('gpurun_out/ab_$1_$2.json').read().strip().splitlines()[-1])['dominance_roofline']; print('ppt $1 r $2', {k: d[k] for k in ('achieved','frac','dominance_ms','ms_per_query','pair_tests_W','skyline_size','sfs_rounds','local_sfs_ms','global_sfs_ms')})"
done
