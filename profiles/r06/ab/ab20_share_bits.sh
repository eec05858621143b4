set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab20
for pass in 1 2; do for b in 11 10 9; do
  PIPELINEDP_AMD_TEST_HOOKS=1 PIPELINEDP_AMD_BUCKET_BITS=$b timeout -k 10 300 python -u bench.py --share-of 8 --no-api --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/ab20/share_b$b.$pass.json 2> gpurun_out/ab20/share_b$b.$pass.err || exit 1
  python3 -c "
import json,sys
r=json.loads([l for l in open('gpurun_out/ab20/share_b$b.$pass.json') if l.startswith('{')][-1])
k=r['kernels']
print('b$b.$pass', round(r['ms_per_step'],3), r['bound_plan']['n_buckets'], {n: round(v['ms']*v.get('launches_per_step',1),3) for n,v in k.items() if v['ms']*v.get('launches_per_step',1)>0.02})
"
done; done
