# round 3: does the flattened kernel's 16-B payload phase cost HBM bytes?  hbmcal's ph_* kernels
# (one wave per SIMD, 1536 contiguous bytes per lane, 64 B per step, spin x 1000 VALU between steps),
# FETCH_SIZE / WRITE_SIZE / EA request passes per kernel, each its own run.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/phase; export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for k in ph_wr_0 ph_wr_16 ph_rd_0 ph_rd_16; do
  for spin in 0 4; do
    o=gpurun_out/phase/${k}_s$spin
    timeout -k 10 60 tools/build/hbmcal $k $spin > $o.time.json || exit 1
    if [ ${k:3:2} = wr ]; then c="WRITE_SIZE"; e="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; else c="FETCH_SIZE"; e="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; fi
    timeout -s KILL 60 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $o.size -o p -- tools/build/hbmcal $k $spin > /dev/null 2>&1 || exit 1
    timeout -s KILL 60 rocprofv3 --pmc $e --kernel-trace --output-format csv -d $o.ea -o p -- tools/build/hbmcal $k $spin > /dev/null 2>&1 || exit 1
    echo "$k spin=$spin $(cat $o.time.json)"
  done
done
python3 tools/pmc_summary.py gpurun_out/phase/* > gpurun_out/phase_summary.txt 2>&1 || true
