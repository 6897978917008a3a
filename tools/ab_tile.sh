set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for rep in 1 2; do
for v in new old; do
  for sh in 0 112; do
    if [ $v = old ]; then L="RG_AEAD_LIB=tools/build/librg_oldtile.so"; else L=""; fi
    env $L timeout -k 10 200 python bench.py --workload cfg4 --frame-shift $sh --steps 20 --warmup 3 --cpu-seconds 0 --no-cold > gpurun_out/ab_${v}_${sh}_$rep.log 2>&1
    python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/ab_${v}_${sh}_$rep.log') if l.startswith('{')][-1]); print('$v', $sh, $rep, d['value'], d['seal_ms'], d['open_ms'])"
  done
done
done
