set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/c4
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
true


for v in 16 32 64; do
  KSQL_AMD_LIB_VARIANT=tune KHIP_PROBE_DPR=$v timeout -k 10 200 python -u bench.py --config clickstream_join --steps 5 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/c4/b$v.jsonl 2>/dev/null || exit 4
  python3 -c "import json; d=json.loads(open('gpurun_out/c4/b$v.jsonl').read()); print('DPR $v', '%.3e'%d['value'], '%.2f ms'%d['ms_per_step'])"
done
