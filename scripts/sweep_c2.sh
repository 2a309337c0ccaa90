set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/sweep
run() { tag=$1; shift; env "$@" timeout -k 10 120 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/sweep/$tag.log 2>&1 || { echo "$tag failed"; tail -5 gpurun_out/sweep/$tag.log; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/sweep/$tag.log') if l.startswith('{')][0]); r=d['roofline']; print('$tag', '%.4g'%d['value'], '%.3f'%r['push_ms'], {k:round(v['ms'],3) for k,v in r['per_kernel'].items()})"; }
run base X=1
run lds120 KHIP_LDS_KB=120
run lds158 KHIP_LDS_KB=158
run tile16 KHIP_TILE_ITEMS=16
run tile64 KHIP_TILE_ITEMS=64
run scat16 KHIP_SCATTER_U=16
run scat4 KHIP_SCATTER_U=4
run p13 KHIP_PART_LOG2=13
