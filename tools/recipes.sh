#!/bin/bash
# tools/recipes.sh NAME [ARGS...] -- the exact command of every measured experiment of rounds 2-5, one
# function each (they were ~90 separate tools/call_*.sh files until round 5: VERDICT r4 item 8).  NAME is
# the old file name without "call_" and ".sh" (call_r4_flat.sh -> r4_flat); the profiles/ record a
# recipe produced names it.  `tools/recipes.sh --list` prints the names with their first comment line.
# Run on the GPU box through gpurun:  gpurun -- bash tools/recipes.sh r4_flat
set -u
SELF=$(readlink -f "$0")
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export HSA_ENABLE_IPC_MODE_LEGACY=0

recipe_ab_lines() {
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 bash tools/ab.sh "base nolines nocur" "cfg2" 3 --no-cold || exit $?
for v in base nolines; do
  if [ $v = base ]; then unset RG_AEAD_LIB; else export RG_AEAD_LIB=tools/build/librg_$v.so; fi
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmcf_$v -o p -- python3 bench.py --workload cfg2 --steps 5 --warmup 2 --cpu-seconds 0 --no-cold > gpurun_out/pmcf_$v.log 2>&1 || exit $?
  timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmcw_$v -o p -- python3 bench.py --workload cfg2 --steps 5 --warmup 2 --cpu-seconds 0 --no-cold > gpurun_out/pmcw_$v.log 2>&1 || exit $?
done
echo done
}

recipe_cfg2_diag() {
# cfg2 diagnostics: per-wave stamps, compute-only / memory-only / store-to-one-block modes, lanes per packet
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 120 python tools/stamps.py --workload cfg2 --plan 0 > gpurun_out/diag_stamps.log 2>&1 || exit $?
tail -n 30 gpurun_out/diag_stamps.log
for v in "base:" "m1:--debug-mode 1 --no-verify" "m2:--debug-mode 2 --no-verify" "m8:--debug-mode 8 --no-verify" "l2:--lanes 2" "p0:--plan 0" "wg2:--wg-per-cu 2 --plan 0"; do
  n=${v%%:*}; f=${v#*:}
  timeout -k 10 120 python bench.py --workload cfg2 --steps 20 --warmup 3 --cpu-seconds 0 --no-cold $f > gpurun_out/diag_$n.log 2>&1 || exit $?
  echo "$n $(grep '^{' gpurun_out/diag_$n.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["seal_ms"], d["open_ms"], d["config"]["kernel"][:50])')"
done
}

recipe_cfg2_diag2() {
# cfg2 diagnostics 2: compute-only / no-store modes at 1 and 2 lanes per packet, stamps at 2 lanes
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for v in "base:--plan 0" "m1:--debug-mode 1 --no-verify --plan 0" "m7:--debug-mode 7 --no-verify --plan 0" "l2:--lanes 2 --plan 0" "l2m1:--lanes 2 --debug-mode 1 --no-verify --plan 0" "l2m7:--lanes 2 --debug-mode 7 --no-verify --plan 0" "l4m1:--lanes 4 --debug-mode 1 --no-verify --plan 0"; do
  n=${v%%:*}; f=${v#*:}
  timeout -k 10 120 python bench.py --workload cfg2 --steps 20 --warmup 3 --cpu-seconds 0 --no-cold $f > gpurun_out/diag2_$n.log 2>&1 || exit $?
  echo "$n $(grep '^{' gpurun_out/diag2_$n.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["seal_ms"], d["open_ms"], d["config"]["kernel"][:50])')"
done
for m in 1 7 0; do
timeout -k 10 120 python tools/stamps.py --workload cfg2 --plan 0 --lanes 2 --mode $m > gpurun_out/diag2_stamps_l2_m$m.log 2>&1 || exit $?
done
timeout -k 10 120 python tools/stamps.py --workload cfg2 --plan 0 --mode 1 > gpurun_out/diag2_stamps_l1_m1.log 2>&1 || exit $?
timeout -k 10 120 python tools/stamps.py --workload cfg2 --plan 0 --mode 7 > gpurun_out/diag2_stamps_l1_m7.log 2>&1 || exit $?
}

recipe_cfg2_diag3() {
# cfg2 diagnostics 3: loads before stores (lf1), two waves per SIMD at 2 lanes per packet
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 bash tools/ab.sh "base lf1 d4 d4lf" "cfg2" 3 --no-cold || exit $?
for v in "l2w2:--lanes 2 --wg-per-cu 2 --plan 0" "l2w2m1:--lanes 2 --wg-per-cu 2 --plan 0 --debug-mode 1 --no-verify" "l2w2m7:--lanes 2 --wg-per-cu 2 --plan 0 --debug-mode 7 --no-verify" "l4w4:--lanes 4 --wg-per-cu 4 --plan 0"; do
  n=${v%%:*}; f=${v#*:}
  timeout -k 10 120 python bench.py --workload cfg2 --steps 20 --warmup 3 --cpu-seconds 0 --no-cold $f > gpurun_out/diag3_$n.log 2>&1 || exit $?
  echo "$n $(grep '^{' gpurun_out/diag3_$n.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["seal_ms"], d["open_ms"], d["config"]["kernel"][:50])')"
done
export RG_AEAD_LIB=tools/build/librg_d4lf.so
timeout -k 10 120 python tools/stamps.py --workload cfg2 --plan 0 --mode 3 > gpurun_out/diag3_stamps_lf1.log 2>&1 || exit $?
}

recipe_cfg2_storecost() {
# cfg2 store cost: default vs mode 8 (line stores to two cache-resident lines per frame) vs mode 7 (no payload stores), with stamps
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for v in "base:" "m8:--debug-mode 8 --no-verify" "m7:--debug-mode 7 --no-verify"; do
  n=${v%%:*}; f=${v#*:}
  timeout -k 10 120 python bench.py --workload cfg2 --steps 20 --warmup 3 --cpu-seconds 0 --no-cold --plan 0 $f > gpurun_out/sc_$n.log 2>&1 || exit $?
  echo "$n $(grep '^{' gpurun_out/sc_$n.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["seal_ms"], d["open_ms"])')"
done
timeout -k 10 120 python tools/stamps.py --workload cfg2 --plan 0 --mode 8 > gpurun_out/sc_stamps_m8.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/sc_stamps_m8.log | python3 -c "
import sys,json; d=json.loads(sys.stdin.read())
for k,v in d.items(): print(k, round(v['cycles_per_wave_mean']), v['wave_us_pct_0_10_50_90_100'], v['shader_clock_ghz'], v['end_us_pct_0_50_90_100'])"
}

recipe_cfg2_tiles() {
# cfg2 on the LDS-staged tile kernel: windows 1/2 x segments 1/2/4, against the automatic choice
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for v in "auto:" "t1s1:--staged 1 --segments 1" "t1s2:--staged 1 --segments 2" "t2s1:--staged 2 --segments 1" "t2s2:--staged 2 --segments 2" "t2s4:--staged 2 --segments 4" "t1s4:--staged 1 --segments 4" "c4auto:--workload cfg4" "c4t2s2:--workload cfg4 --staged 2 --segments 2"; do
  n=${v%%:*}; f=${v#*:}
  w=cfg2; case "$f" in *cfg4*) w=cfg4; f=${f/--workload cfg4/};; esac
  timeout -k 10 120 python bench.py --workload $w --steps 20 --warmup 3 --cpu-seconds 0 --no-cold $f > gpurun_out/tiles_$n.log 2>&1 || exit $?
  echo "$n $(grep '^{' gpurun_out/tiles_$n.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["seal_ms"], d["open_ms"], d["config"]["kernel"][:60])')"
done
}

recipe_cfg2_wt() {
# cfg2: write-through ring stores (wt1) against the default build
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
RG_AEAD_LIB=tools/build/librg_wt1.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "full_config_digest or random_batches or open_failures or reference_framed" --timeout 120 --timeout-method thread > gpurun_out/wt_pytest.log 2>&1; rc=$?; tail -n 3 gpurun_out/wt_pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 bash tools/ab.sh "base wt1" "cfg2" 3 --no-cold || exit $?
export RG_AEAD_LIB=tools/build/librg_wt1.so
timeout -k 10 120 python tools/stamps.py --workload cfg2 --plan 0 --mode 3 > gpurun_out/wt_stamps.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmcw_wt1 -o p -- python3 bench.py --workload cfg2 --steps 5 --warmup 2 --cpu-seconds 0 --no-cold > gpurun_out/pmcw_wt1.log 2>&1 || exit $?
}

recipe_cfg3_stamps() {
# cfg3: flattened kernel phase stamps with wall-clock start/end, and the bench line
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 120 python tools/flat_stamps.py --workload cfg3 > gpurun_out/flat_stamps.log 2>&1 || exit $?
cat gpurun_out/flat_stamps.log | grep -v amdgpu.ids
timeout -k 10 120 python bench.py --workload cfg3 --steps 20 --warmup 3 --cpu-seconds 0 --no-cold > gpurun_out/cfg3_bench.log 2>&1 || exit $?
grep '^{' gpurun_out/cfg3_bench.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["seal_ms"], d["open_ms"])'
}

recipe_cfg3_tiles() {
# cfg3 on the tile kernel (dynamic deal) against the automatic choice (flattened)
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for v in "auto:" "t2:--staged 2" "t1:--staged 1" "t2s1:--staged 2 --segments 1" "t2s2:--staged 2 --segments 2" "pipe:--staged 0"; do
  n=${v%%:*}; f=${v#*:}
  timeout -k 10 120 python bench.py --workload cfg3 --steps 20 --warmup 3 --cpu-seconds 0 --no-cold --forged 0 $f > gpurun_out/c3t_$n.log 2>&1 || exit $?
  echo "$n $(grep '^{' gpurun_out/c3t_$n.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["seal_ms"], d["open_ms"], d["config"]["kernel"][:60])')"
done
}

recipe_cfg4_stamps() {
# cfg4: tile kernel section stamps
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 200 python tools/stamps.py --workload cfg4 > gpurun_out/cfg4_stamps.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/cfg4_stamps.log
}

recipe_check_bench() {
# quick check of the bench line fields (wire rate, copy ceiling) and smoke
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -n 1 gpurun_out/smoke.log
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --cpu-seconds 0 > gpurun_out/chk_cfg2.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --workload cfg5 --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/chk_cfg5.log 2>&1 || exit $?
for f in gpurun_out/chk_cfg2.log gpurun_out/chk_cfg5.log; do grep '^{' $f | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["wire_gib_s"], d["roofline"])'; done
}

recipe_flat_npf() {
# flat kernel next-packet prefetch: flat GPU tests, A/B on cfg3, stamps
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "flat or auto or digest or malformed or keepalive" --timeout 120 --timeout-method thread > gpurun_out/npf_pytest.log 2>&1; rc=$?; tail -n 3 gpurun_out/npf_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 bash tools/ab.sh "base npf0" "cfg3" 4 --no-cold || exit $?
timeout -k 10 120 python tools/flat_stamps.py --workload cfg3 > gpurun_out/flat_stamps_npf.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/flat_stamps_npf.log | cut -c1-420
}

recipe_flat_perwave() {
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 120 python tools/flat_stamps.py --workload cfg3 --per-wave > gpurun_out/flat_perwave.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/flat_perwave.log | tail -n 3 | cut -c1-1500
}

recipe_flat_quad() {
# flat kernel quad-lane overflow key blocks: GPU tests, A/B on cfg3, stamps
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/quad_pytest.log 2>&1; rc=$?; tail -n 3 gpurun_out/quad_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 bash tools/ab.sh "base quad0" "cfg3" 4 --no-cold || exit $?
timeout -k 10 120 python tools/flat_stamps.py --workload cfg3 > gpurun_out/flat_stamps_quad.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/flat_stamps_quad.log | cut -c1-700
}

recipe_forged() {
# forged-tag open cost on the final build (cfg2 pipelined, cfg4 tiles)
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for v in "cfg2:0.1" "cfg2:1.0" "cfg4:0.1" "cfg4:1.0"; do
  w=${v%%:*}; f=${v#*:}
  timeout -k 10 200 python bench.py --workload $w --steps 10 --warmup 2 --cpu-seconds 0 --no-cold --forged $f > gpurun_out/forged_${w}_$f.log 2>&1 || exit $?
  echo "$w $f $(grep '^{' gpurun_out/forged_${w}_$f.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["open_ms"], d["forged_open"])')"
done
}

recipe_r3_abl() {
# round 3, config 2: seal with the line stores dropped (abl1) / the LDS ring dropped (abl2) against the default build
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
bash tools/ab.sh "base abl1 abl2" cfg2 2 --no-cold --no-verify || exit $?
for v in base abl1 abl2; do
  if [ $v = base ]; then unset RG_AEAD_LIB; else export RG_AEAD_LIB=tools/build/librg_$v.so; fi
  timeout -k 10 120 python tools/stamps.py --workload cfg2 --plan 0 > gpurun_out/abl_st_$v.json 2>&1 || exit $?
  echo "== $v stamps"
  grep -A1 cycles_per_wave gpurun_out/abl_st_$v.json | head -2
done
}

recipe_r3_coop() {
# round 3, config 3: workgroup-cooperative unit search over 4096-packet groups (default: work = 1 + 8 x chunks;
# coopw1: 1 + chunks; nocoop: the one-wave search over 1024-packet groups).  Flat-kernel tests, then A/B + phase stamps.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_forged.py -x -q -k "flat or imix or digest or coop" --timeout 120 --timeout-method thread > gpurun_out/coop_tests.log 2>&1
rc=$?; tail -3 gpurun_out/coop_tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab.sh "nocoop base" cfg3 3 --no-cold --forged 0 || exit $?
for v in nocoop base; do
  if [ $v = base ]; then unset RG_AEAD_LIB; else export RG_AEAD_LIB=tools/build/librg_$v.so; fi
  timeout -k 10 120 python tools/flat_stamps.py --workload cfg3 > gpurun_out/coop_st_$v.log 2>&1 || exit $?
  echo "== $v"; grep -v amdgpu.ids gpurun_out/coop_st_$v.log | cut -c1-600
done
}

recipe_r3_coop2() {
# round 3, config 3: the workgroup-cooperative unit search (base) against the one-wave search (nocoop), 5 interleaved reps
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "coop or digest" --timeout 120 --timeout-method thread > gpurun_out/coop2_tests.log 2>&1
rc=$?; tail -1 gpurun_out/coop2_tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab.sh "nocoop base" cfg3 5 --no-cold --forged 0
}

recipe_r3_coop3() {
# round 3, config 3: cooperative search with float targets and only in-range boundary counts; tests, A/B vs nocoop, stamps
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_forged.py -x -q -k "flat or imix or digest or coop" --timeout 120 --timeout-method thread > gpurun_out/coop3_tests.log 2>&1
rc=$?; tail -1 gpurun_out/coop3_tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab.sh "nocoop base" cfg3 4 --no-cold --forged 0 || exit $?
timeout -k 10 120 python tools/flat_stamps.py --workload cfg3 > gpurun_out/coop3_st.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/coop3_st.log | cut -c1-420
}

recipe_r3_coop4() {
# round 3, config 3: cooperative search staging its first sub-units from a shared LDS window (base) vs from memory (prev)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_forged.py -x -q -k "flat or imix or digest or coop" --timeout 120 --timeout-method thread > gpurun_out/coop4_tests.log 2>&1
rc=$?; tail -1 gpurun_out/coop4_tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab.sh "prev base" cfg3 4 --no-cold --forged 0 || exit $?
timeout -k 10 120 python tools/flat_stamps.py --workload cfg3 > gpurun_out/coop4_st.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/coop4_st.log | cut -c1-420
}

recipe_r3_dma() {
# round 3: the staged (LDS-DMA) chunk stream of the pipelined kernel on config 2 -- per-wave stamps with
# and without it, interleaved A/B of staging depths, forged-tag open cost
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 120 python tools/stamps.py --workload cfg2 --plan 0 > gpurun_out/r3_stamps_dma.log 2>&1 || exit $?
RG_AEAD_LIB=tools/build/librg_nodma.so timeout -k 10 120 python tools/stamps.py --workload cfg2 --plan 0 > gpurun_out/r3_stamps_nodma.log 2>&1 || exit $?
grep -A3 '"seal"\|"open"' gpurun_out/r3_stamps_dma.log gpurun_out/r3_stamps_nodma.log | grep -v "^--$" | head -20
tools/ab.sh "base nodma d3 d6" "cfg2" 2 --no-cold || exit $?
for f in 0.01 0.1; do
  timeout -k 10 120 python bench.py --steps 10 --warmup 3 --no-cold --cpu-seconds 0 --forged $f > gpurun_out/r3_forged_$f.log 2>&1 || exit $?
  echo "forged $f $(grep '^{' gpurun_out/r3_forged_$f.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["open_ms"], d["forged_open"])')"
done
timeout -k 10 120 python bench.py --workload cfg4 --steps 5 --warmup 2 --no-cold --cpu-seconds 0 --forged 0.1 > gpurun_out/r3_forged_cfg4.log 2>&1 || exit $?
echo "cfg4 forged 0.1 $(grep '^{' gpurun_out/r3_forged_cfg4.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["open_ms"], d["forged_open"])')"
}

recipe_r3_final() {
# round 3: what the driver runs at round end, on the final build -- every GPU test, smoke(), the default bench line
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/final_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/final_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/final_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/final_bench.log 2>&1 || exit $?
grep '^{' gpurun_out/final_bench.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["seal_ms"], d["open_ms"], d["roofline"]["frac"], d["valu_roofline"]["frac"], [f["ratio"] for f in d["forged_open"]])'
}

recipe_r3_flatforged() {
# round 3: the flat kernel's cooperative restore -- forged-frame tests, flat parity, forged-open cost on config 3
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_forged.py tests/test_gpu_parity.py -k "forged or flat or untouched or imix" -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_flat_tests.log 2>&1; rc=$?
tail -n 3 gpurun_out/r3_flat_tests.log
[ $rc -eq 0 ] || exit $rc
for f in 0.01 0.1 1.0; do
  timeout -k 10 150 python bench.py --workload cfg3 --steps 5 --warmup 2 --no-cold --cpu-seconds 0 --forged $f > gpurun_out/r3f_cfg3_$f.log 2>&1 || exit $?
  echo "cfg3 $f $(grep '^{' gpurun_out/r3f_cfg3_$f.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["open_ms"], d["forged_open"])')"
done
}

recipe_r3_flattraffic() {
# round 3: where config 3's extra HBM bytes come from -- FETCH_SIZE / WRITE_SIZE of the flattened kernel
# in the in-tree build and in the no-payload-store / no-payload-load ablations (output invalid there)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/ft; export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for v in ${VS:-base nostore noload}; do
  if [ $v = base ]; then unset RG_AEAD_LIB; else export RG_AEAD_LIB=tools/build/librg_$v.so; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/ft/${v}_$c -o p -- \
      python3 bench.py --workload ${W:-cfg3} --steps 5 --warmup 2 --cpu-seconds 0 --no-cold --forged 0 --no-graph > gpurun_out/ft/${v}_$c.log 2>&1
    rc=$?; [ $rc -gt 1 ] && exit $rc  # the ablations fail the bench's final open check (rc 1): counters are in
  done
done
python3 tools/pmc_summary.py gpurun_out/ft/* > gpurun_out/ft_summary.txt 2>&1 || true
}

recipe_r3_forged() {
# round 3: forged-tag open cost with the corrected harness (clean and forged opens both behind a spin kernel),
# default (decrypt + cooperative restore) and verify-then-decrypt (mf) builds; configs 2, 3, 4
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for lib in base mf; do
  if [ $lib = base ]; then unset RG_AEAD_LIB; else export RG_AEAD_LIB=tools/build/librg_$lib.so; fi
  for w in cfg2 cfg3 cfg4; do
    for f in 0.01 0.1 1.0; do
      timeout -k 10 150 python bench.py --workload $w --steps 5 --warmup 2 --no-cold --cpu-seconds 0 --forged $f > gpurun_out/r3f_${lib}_${w}_$f.log 2>&1 || exit $?
      echo "$lib $w $f $(grep '^{' gpurun_out/r3f_${lib}_${w}_$f.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["open_ms"], d["forged_open"])')"
    done
  done
done
}

recipe_r3_lds() {
# round 3: LDS counters of the transport kernels (config 2 pipelined ring, config 3 flattened, config 4 tiles):
# bank-conflict and unaligned-stall cycles against all LDS-array cycles; one pass per workload
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/lds; export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for W in ${WS:-cfg2 cfg3 cfg4}; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT \
      SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAVES --kernel-trace --output-format csv -d gpurun_out/lds/${TAG:-base}_$W -o p -- \
      python3 bench.py --workload $W --steps 5 --warmup 2 --cpu-seconds 0 --no-cold --forged 0 --no-graph > gpurun_out/lds/${TAG:-base}_$W.log 2>&1 || exit 1
done
python3 tools/pmc_summary.py gpurun_out/lds/* > gpurun_out/lds_summary.txt 2>&1 || true
}

recipe_r3_macfirst() {
# round 3: verify-then-decrypt open (RG_PIPE_MAC_FIRST) -- forged/parity tests, forged-tag open cost,
# interleaved A/B against decrypt-first (df) and staggered wave starts
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_forged.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_mf_tests.log 2>&1; rc=$?
tail -n 3 gpurun_out/r3_mf_tests.log
[ $rc -eq 0 ] || exit $rc
for f in 0.01 0.1 1.0; do
  timeout -k 10 120 python bench.py --steps 10 --warmup 3 --no-cold --cpu-seconds 0 --forged $f > gpurun_out/r3_forged_$f.log 2>&1 || exit $?
  echo "cfg2 forged $f $(grep '^{' gpurun_out/r3_forged_$f.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["open_ms"], d["forged_open"])')"
done
tools/ab.sh "base df stag16 stag32" "cfg2" 3 --no-cold || exit $?
}

recipe_r3_nolines() {
# round 3: config 2 without the LDS ring (lane-per-frame 64-byte frame-aligned stores), with and without the
# next chunk's loads issued ahead of the step's stores; parity of the pipelined paths on each build, then A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for V in nolines nolineslf; do
  RG_AEAD_LIB=tools/build/librg_$V.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_forged.py -x -q -k "pipe or cfg2 or auto" --timeout 120 --timeout-method thread > gpurun_out/${V}_tests.log 2>&1
  rc=$?; tail -1 gpurun_out/${V}_tests.log; [ $rc -ne 0 ] && exit $rc
done
bash tools/ab.sh "base nolines nolineslf" "cfg2" 3 --no-cold --forged 0
}

recipe_r3_ntload() {
# round 3: streaming (nt) payload loads in the flattened kernel -- do the partially written lines survive
# longer in L2 (config 3 WRITE_SIZE), and what does it do to the launch?  Parity on the variant first.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
RG_AEAD_LIB=tools/build/librg_ntload.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "flat" --timeout 120 --timeout-method thread > gpurun_out/nt_tests.log 2>&1
rc=$?; tail -2 gpurun_out/nt_tests.log; [ $rc -ne 0 ] && exit $rc
VS="ntload" bash tools/recipes.sh r3_flattraffic || exit 1
bash tools/ab.sh "base ntload" "cfg3" 3 --no-cold --forged 0
}

recipe_r3_phase() {
# round 3: does the flattened kernel's 16-B payload phase cost HBM bytes?  hbmcal's ph_* kernels
# (one wave per SIMD, 1536 contiguous bytes per lane, 64 B per step, spin x 1000 VALU between steps),
# FETCH_SIZE / WRITE_SIZE / EA request passes per kernel, each its own run.
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
}

recipe_r3_quad() {
# round 3: quad-transposed block stores (no LDS ring) in the pipelined kernel's uniform waves: parity + forged tests,
# then interleaved A/B against the LDS-ring build (ring = -DRG_PIPE_QUAD=0) and per-wave cycles
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 700 python -u -m pytest tests/test_gpu_forged.py tests/test_gpu_parity.py tests/test_gpu_sessions.py tests/test_gpu_sessions_dev.py -x -q --timeout 120 --timeout-method thread > gpurun_out/quad_tests.log 2>&1
rc=$?; tail -3 gpurun_out/quad_tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab.sh "ring base" cfg2 3 --no-cold --forged 0 || exit $?
for v in ring base; do
  if [ $v = base ]; then unset RG_AEAD_LIB; else export RG_AEAD_LIB=tools/build/librg_$v.so; fi
  timeout -k 10 120 python tools/stamps.py --workload cfg2 --plan 0 > gpurun_out/q_st_$v.json 2>&1 || exit $?
  echo "== $v $(python3 -c "import json; t=open('gpurun_out/q_st_$v.json').read(); d=json.loads(t[t.index('{'):]); print(d['seal']['cycles_per_wave_mean'], d['seal']['end_us_pct_0_50_90_100'], d['open']['cycles_per_wave_mean'], d['open']['end_us_pct_0_50_90_100'])")"
done
}

recipe_r3_rehearse() {
# round 3: GPU tests on the current build, then the N > 1 bench path rehearsed on one GPU (2 ranks sharing it)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/allgpu.log 2>&1
rc=$?; tail -2 gpurun_out/allgpu.log; [ $rc -ne 0 ] && exit $rc
RG_BENCH_SHARE_GPU=1 timeout -k 10 400 python bench.py --gpus 2 --steps 5 --warmup 2 --cpu-seconds 2 > gpurun_out/rehearse2.log 2>&1
rc=$?; tail -c 3000 gpurun_out/rehearse2.log; exit $rc
}

recipe_r3_rehearse_torchrun() {
# round 3: the N > 1 bench path rehearsed on one GPU exactly as the driver launches it (torch.distributed.run,
# WORLD_SIZE set, bench.py does not spawn ranks itself); 2 ranks then 4 ranks sharing the GPU over gloo
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for n in 2 4; do
  RG_BENCH_SHARE_GPU=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 5 --warmup 2 --cpu-seconds 2 \
    > gpurun_out/rehearse_tr$n.log 2>&1
  rc=$?; grep '^{' gpurun_out/rehearse_tr$n.log | cut -c1-400; [ $rc -ne 0 ] && { tail -20 gpurun_out/rehearse_tr$n.log; exit $rc; }
done
exit 0
}

recipe_r3_sc1() {
# round 3: write-through (sc1) frame stores -- pipelined kernel's line-store waves through a buffer window, tile
# kernel's window stores.  Parity + forged-frame tests on the new build, then interleaved A/B:
# old = previous commit (plain stores), nosc1 = new code with RG_STORE_SC1=0, base = new (sc1)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_forged.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sc1_tests.log 2>&1
rc=$?; tail -3 gpurun_out/sc1_tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab.sh "old nosc1 base" "cfg2 cfg3 cfg4 cfg5" 2 --no-cold --forged 0
}

recipe_r3_spread() {
# round 3: forged-frame restore with wavefront-scope ordering (tests + open cost), and config-2
# experiments against the lockstep memory bursts: line stores spread over the rounds, staggered wave starts
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_forged.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_forged_tests.log 2>&1; rc=$?
tail -n 3 gpurun_out/r3_forged_tests.log
[ $rc -le 1 ] || exit $rc
for f in 0.01 0.1 1.0; do
  timeout -k 10 120 python bench.py --steps 10 --warmup 3 --no-cold --cpu-seconds 0 --forged $f > gpurun_out/r3_forged_$f.log 2>&1 || exit $?
  echo "cfg2 forged $f $(grep '^{' gpurun_out/r3_forged_$f.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["open_ms"], d["forged_open"])')"
done
for f in 0.01 0.1; do
  timeout -k 10 120 python bench.py --workload cfg4 --steps 5 --warmup 2 --no-cold --cpu-seconds 0 --forged $f > gpurun_out/r3_forged_cfg4_$f.log 2>&1 || exit $?
  echo "cfg4 forged $f $(grep '^{' gpurun_out/r3_forged_cfg4_$f.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["open_ms"], d["forged_open"])')"
done
tools/ab.sh "base spread wt3 stag16 stag5" "cfg2" 2 --no-cold || exit $?
}

recipe_r3_spread2() {
# round 3, config 2: line stores spread over the keystream rounds (compiler-visible buffer stores) and lane-per-frame
# stores without the ring (nolines) against the default build; interleaved A/B + per-wave cycles
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
bash tools/ab.sh "base spread nolines" cfg2 3 --no-cold --forged 0 || exit $?
for v in base spread nolines; do
  if [ $v = base ]; then unset RG_AEAD_LIB; else export RG_AEAD_LIB=tools/build/librg_$v.so; fi
  timeout -k 10 120 python tools/stamps.py --workload cfg2 --plan 0 > gpurun_out/sp_st_$v.json 2>&1 || exit $?
  echo "== $v $(python3 -c "import json; t=open('gpurun_out/sp_st_$v.json').read(); d=json.loads(t[t.index('{'):]); print(d['seal']['cycles_per_wave_mean'], d['seal']['end_us_pct_0_50_90_100'], d['open']['cycles_per_wave_mean'])")"
done
}

recipe_r3_variant() {
# round 3: one flattened-kernel build variant (tools/build/librg_$V.so): parity of the flat paths and the
# forged-frame tests on it, config-3 FETCH_SIZE / WRITE_SIZE passes, then an interleaved A/B against the
# in-tree build.   usage: V=align bash tools/recipes.sh r3_variant
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
RG_AEAD_LIB=tools/build/librg_$V.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_forged.py -x -q -k "flat or imix or cfg3" --timeout 120 --timeout-method thread > gpurun_out/${V}_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${V}_tests.log; [ $rc -ne 0 ] && exit $rc
[ "${TRAFFIC:-1}" = 1 ] && { VS="base $V" bash tools/recipes.sh r3_flattraffic || exit 1; }
[ "${LDS:-0}" = 1 ] && { RG_AEAD_LIB=tools/build/librg_$V.so TAG=$V WS=cfg3 bash tools/recipes.sh r3_lds || exit 1; }
bash tools/ab.sh "base $V" "${WS:-cfg3}" ${REPS:-3} --no-cold --forged 0
}

recipe_r3_wst() {
# round 3: config-2 step cycles of the pipelined kernel by unrolled position, and the time in an exact vmcnt(16) wait
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
RG_AEAD_LIB=tools/build/librg_wst.so timeout -k 10 120 python tools/wstamps.py > gpurun_out/wst.json 2>gpurun_out/wst.err || exit $?
cat gpurun_out/wst.json
RG_AEAD_LIB=tools/build/librg_wst.so timeout -k 10 120 python tools/wstamps.py --mode 7 > gpurun_out/wst_m7.json 2>&1 || exit $?
echo "== m7"; cat gpurun_out/wst_m7.json
}

recipe_r4_ab() {
# Round 4: config 2 against the round-3 pipelined kernel (tools/build/librg_r3pipe.so), config 3 against two
# flattened-kernel variants (flat2w: 64-packet sub-units and two workgroups = two waves per SIMD;
# flatpk64: 64-packet sub-units alone), and the host-memory path by pipeline slice size (tools/e2e_probe.py).
bash tools/ab.sh "base r3pipe" "cfg2" 3 --no-cold --forged 0 &&
bash tools/ab.sh "base flat2w flatpk64" "cfg3" 3 --no-cold --forged 0 &&
timeout -k 10 300 python tools/e2e_probe.py cfg2 2,4,8,16,32 > gpurun_out/r4_e2e_probe.jsonl && cat gpurun_out/r4_e2e_probe.jsonl
}

recipe_r4_ab2() {
# Round 4: config 3 with two waves per SIMD at 128-packet sub-units (flat2w128: -DRG_FLAT_WG_PER_CU=2, the
# LDS image trimmed to fit two workgroups per CU), and a copy/kernel timeline of the host-memory path
# (rocprofv3 memory-copy + kernel traces of tools/e2e_probe.py at 16 MiB slices).
bash tools/ab.sh "base flat2w128" "cfg3" 3 --no-cold --forged 0 &&
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r4_e2e_trace -o e2e -- python3 tools/e2e_probe.py cfg2 16 > gpurun_out/r4_e2e_trace.log 2>&1
ls -R gpurun_out/r4_e2e_trace | head -20
}

recipe_r4_check() {
# Round 4: GPU tests on the current build, the host-link ceilings (tools/pcie.hip), then config 2 against
# the round-3 pipelined kernel (tools/build/librg_r3pipe.so: commit e1c0e7c's rg_pipe.hip with today's
# other objects) and config 3 against two flattened-kernel variants (flat2w: 64-packet sub-units, two
# workgroups = two waves per SIMD; flatpk64: 64-packet sub-units alone).
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4_gputest.log 2>&1
rc=$?
tail -3 gpurun_out/r4_gputest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 tools/build/pcie 256 > gpurun_out/r4_pcie.json && cat gpurun_out/r4_pcie.json &&
bash tools/ab.sh "base r3pipe" "cfg2" 3 --no-cold --forged 0 &&
bash tools/ab.sh "base flat2w flatpk64" "cfg3" 3 --no-cold --forged 0
}

recipe_r4_check2() {
# Round 4, after the host-path changes: every GPU test, smoke(), and the default bench line (with --e2e).
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4_check2_gputest.log 2>&1
rc=$?
tail -2 gpurun_out/r4_check2_gputest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4_check2_smoke.log 2>&1 && tail -1 gpurun_out/r4_check2_smoke.log &&
timeout -k 10 400 python bench.py --e2e > gpurun_out/r4_check2_default.jsonl 2> gpurun_out/r4_check2_default.err && cut -c1-300 gpurun_out/r4_check2_default.jsonl
}

recipe_r4_check3() {
# Round 4, final build (tile whole-chunk loops, flat carry top bit): every GPU test, smoke(), and the default bench line (with --e2e).
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4_check3_gputest.log 2>&1
rc=$?
tail -2 gpurun_out/r4_check3_gputest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4_check3_smoke.log 2>&1 && tail -1 gpurun_out/r4_check3_smoke.log &&
timeout -k 10 400 python bench.py --e2e > gpurun_out/r4_check3_default.jsonl 2> gpurun_out/r4_check3_default.err && cut -c1-300 gpurun_out/r4_check3_default.jsonl
}

recipe_r4_cores() {
# Round 4: per-wave HW_ID stamps of config 2's seal on the __launch_bounds__(256, 2) build
# (tools/build_variant.sh lb2 -DRG_PIPE_LB2): two lanes per packet, two workgroups per CU.
export RG_AEAD_LIB=tools/build/librg_lb2.so
timeout -k 10 120 python tools/coresidency.py --lanes 2 --wg-per-cu 2 --mode 3 > gpurun_out/r4_cores_l2w2.json &&
timeout -k 10 120 python tools/coresidency.py --lanes 2 --wg-per-cu 2 --mode 1 > gpurun_out/r4_cores_l2w2_m1.json &&
timeout -k 10 120 python tools/coresidency.py --lanes 1 --wg-per-cu 1 --mode 3 > gpurun_out/r4_cores_l1w1.json &&
timeout -k 10 120 python tools/coresidency.py --lanes 1 --wg-per-cu 1 --mode 1 > gpurun_out/r4_cores_l1w1_m1.json
}

recipe_r4_default() {
# Round 4: the default bench line exactly as the driver runs it (no flags; the host path now on by default).
t0=$(date +%s)
timeout -k 10 400 python bench.py > gpurun_out/r4_default_noflags.jsonl 2> gpurun_out/r4_default_noflags.err
rc=$?
echo "wall $(( $(date +%s) - t0 )) s, rc $rc"
python3 -c "import json; d=json.loads(open('gpurun_out/r4_default_noflags.jsonl').read().strip().splitlines()[-1]); print(d['value'], d.get('e2e'))"
exit $rc
}

recipe_r4_defprof() {
# Round 4: rocprofv3 kernel stats of the default bench command itself (python bench.py, no flags).
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_default -o run -- python3 bench.py > gpurun_out/prof_default.log 2>&1
rc=$?
grep '^{' gpurun_out/prof_default.log | cut -c1-200
find gpurun_out/prof_default -name "*kernel_stats.csv" | head -2
exit $rc
}

recipe_r4_e2e() {
# Round 4: the host-memory path with one upload, one kernel and one download stream per context (the
# slices of a direction back to back, the two directions beside each other): the host-path GPU tests,
# the slice-size probe, and a copy/kernel timeline.
timeout -k 10 600 python -u -m pytest tests/test_gpu_sessions.py tests/test_gpu_group.py tests/test_gpu_sessions_dev.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4_e2e_tests.log 2>&1
rc=$?
tail -2 gpurun_out/r4_e2e_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/e2e_probe.py cfg2 4,8,16,32 > gpurun_out/r4_e2e_probe2.jsonl && cat gpurun_out/r4_e2e_probe2.jsonl &&
timeout -k 10 120 tools/build/pcie 256 &&
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r4_e2e_trace2 -o e2e -- python3 tools/e2e_probe.py cfg2 16 > gpurun_out/r4_e2e_trace2.log 2>&1
}

recipe_r4_e2etrace() {
# Round 4: copy + kernel timeline of the host path (config 2, 8 MiB slices), to find where a seal call
# loses to the duplex ceiling (tools/e2e_timeline.py reads the CSVs).
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/e2etrace -o run -- python3 tools/e2e_probe.py cfg2 8 > gpurun_out/e2etrace.log 2>&1
rc=$?
tail -3 gpurun_out/e2etrace.log
find gpurun_out/e2etrace -name "*.csv" | head
exit $rc
}

recipe_r4_e2etrace3() {
# Round 4: host path (config 2, 8 MiB slices) with the HIP API trace beside copies and kernels, to see
# which host call waits (tools/e2e_timeline.py + the api CSV).
timeout -k 10 240 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/e2etrace3 -o run -- python3 tools/e2e_probe.py cfg2 8 > gpurun_out/e2etrace3.log 2>&1
}

recipe_r4_evdev() {
# Round 4: host path with ev_in and ev_run with a device-scope release (hipEventReleaseToDevice) (working tree)
# against the committed build (tools/build/librg_head.so): host-path GPU tests, interleaved
# tools/e2e_probe.py on configs 2 and 3, then a copy + kernel trace of the working tree.
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "host or group or sessions or pinned" --timeout 120 --timeout-method thread > gpurun_out/r4_evdev_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r4_evdev_tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
    for v in head base; do
        if [ "$v" = base ]; then unset RG_AEAD_LIB; else export RG_AEAD_LIB=tools/build/librg_$v.so; fi
        for w in cfg2 cfg3; do
            echo "== $v $w run $r"
            timeout -k 10 240 python tools/e2e_probe.py $w 4,8,16 || exit $?
        done
    done
done 2>&1 | tee gpurun_out/r4_e2e_evdev_ab.txt
unset RG_AEAD_LIB
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/e2etrace6 -o run -- python3 tools/e2e_probe.py cfg2 8 > gpurun_out/e2etrace6.log 2>&1
}

recipe_r4_final() {
# Round 4 final check, as the driver runs it: every GPU test, smoke(), the default bench line; then the
# round's profile set again (kernel stats, FETCH/WRITE, VALU counters, bench rows) on the final build.
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4_final_gputest.log 2>&1
rc=$?
tail -2 gpurun_out/r4_final_gputest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4_final_smoke.log 2>&1 && tail -1 gpurun_out/r4_final_smoke.log &&
bash tools/round_profiles.sh > gpurun_out/r4_final_profiles.log 2>&1 && tail -8 gpurun_out/r4_final_profiles.log
}

recipe_r4_flat() {
# Round 4: flattened-kernel changes (every packet >= 1 chunk step, no skip loops; the stream's first column
# round read from LDS at a packet switch; the last chunk's Horner blocks interleaved with the carry powers;
# descriptor fields kept in registers and counters loaded with them): the flat / forged parity tests, an
# interleaved A/B against the committed build (tools/build_rev.sh head) on config 3 and config 2, the new
# build's cfg3 stamps (diag build), and the host path by slice size again.
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_forged.py -x -q -m gpu \
    -k "flat or open_failures or bad_descriptors or malformed or digest or auto" --timeout 300 --timeout-method thread \
    > gpurun_out/r4_flat_tests.log 2>&1
rc=$?
tail -2 gpurun_out/r4_flat_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/ab.sh "base head" "cfg3" 3 --no-cold --forged 0 &&
bash tools/ab.sh "base head" "cfg2" 1 --no-cold --forged 0 &&
RG_AEAD_LIB=tools/build/librg_diag.so timeout -k 10 200 python tools/flat_stamps.py --workload cfg3 > gpurun_out/r4_cfg3_flat_stamps4.txt 2>&1 && cat gpurun_out/r4_cfg3_flat_stamps4.txt &&
timeout -k 10 300 python tools/e2e_probe.py cfg2 8,16,32 > gpurun_out/r4_e2e_probe6.jsonl && cat gpurun_out/r4_e2e_probe6.jsonl
}

recipe_r4_full() {
# Round 4: every GPU test, the host-memory path by slice size (four slots), the default bench line, the
# single-process bench on one GPU (two contexts sharing it: a rehearsal), and the N = 2 launcher path as
# the driver runs it, both ranks sharing the GPU (RG_BENCH_SHARE_GPU=1; gloo bookkeeping).
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4_gputest.log 2>&1
rc=$?
tail -2 gpurun_out/r4_gputest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/e2e_probe.py cfg2 8,16,32 > gpurun_out/r4_e2e_probe3.jsonl && cat gpurun_out/r4_e2e_probe3.jsonl &&
timeout -k 10 400 python bench.py --e2e > gpurun_out/r4_bench_default.jsonl 2> gpurun_out/r4_bench_default.err && cat gpurun_out/r4_bench_default.jsonl &&
RG_BENCH_SHARE_GPU=1 timeout -k 10 300 python bench.py --single-process --gpus 2 --steps 5 --warmup 2 > gpurun_out/r4_single_share2.jsonl 2> gpurun_out/r4_single_share2.err && cat gpurun_out/r4_single_share2.jsonl &&
RG_BENCH_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --cpu-seconds 2 > gpurun_out/r4_rehearse_torchrun2.jsonl 2> gpurun_out/r4_rehearse_torchrun2.err && cat gpurun_out/r4_rehearse_torchrun2.jsonl
RG_AEAD_LIB=tools/build/librg_diag.so timeout -k 10 200 python tools/flat_stamps.py --workload cfg3 > gpurun_out/r4_cfg3_flat_stamps.txt 2>&1 && cat gpurun_out/r4_cfg3_flat_stamps.txt
}

recipe_r4_hostload() {
# Round 4: host path with uploads read by a 128-workgroup host-load kernel (working tree)
# against the committed build (tools/build/librg_head.so): host-path GPU tests, interleaved
# tools/e2e_probe.py on configs 2 and 3, then a copy + kernel trace of the working tree.
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "host or group or sessions or pinned" --timeout 120 --timeout-method thread > gpurun_out/r4_hostload_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r4_hostload_tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
    for v in head base; do
        if [ "$v" = base ]; then unset RG_AEAD_LIB; else export RG_AEAD_LIB=tools/build/librg_$v.so; fi
        for w in cfg2 cfg3; do
            echo "== $v $w run $r"
            timeout -k 10 240 python tools/e2e_probe.py $w 4,8,16 || exit $?
        done
    done
done 2>&1 | tee gpurun_out/r4_e2e_hostload_ab.txt
unset RG_AEAD_LIB
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/e2etrace8 -o run -- python3 tools/e2e_probe.py cfg2 8 > gpurun_out/e2etrace8.log 2>&1
}

recipe_r4_hoststore() {
# Round 4: host path with downloads written by a 64-workgroup host-store kernel (working tree)
# against the committed build (tools/build/librg_head.so): host-path GPU tests, interleaved
# tools/e2e_probe.py on configs 2 and 3, then a copy + kernel trace of the working tree.
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "host or group or sessions or pinned" --timeout 120 --timeout-method thread > gpurun_out/r4_hoststore_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r4_hoststore_tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
    for v in head base; do
        if [ "$v" = base ]; then unset RG_AEAD_LIB; else export RG_AEAD_LIB=tools/build/librg_$v.so; fi
        for w in cfg2 cfg3; do
            echo "== $v $w run $r"
            timeout -k 10 240 python tools/e2e_probe.py $w 4,8,16 || exit $?
        done
    done
done 2>&1 | tee gpurun_out/r4_e2e_hoststore_ab.txt
unset RG_AEAD_LIB
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/e2etrace5 -o run -- python3 tools/e2e_probe.py cfg2 8 > gpurun_out/e2etrace5.log 2>&1
}

recipe_r4_hwq() {
# Round 4 diagnostic: the host path (config 2) with 4 (the box's default), 8 and 16 hardware queues per
# process, to see whether the pipeline streams share a queue.
for q in 4 8 16; do
    echo "== GPU_MAX_HW_QUEUES=$q"
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python tools/e2e_probe.py cfg2 8,16 || exit $?
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r4_e2e_hwq.txt
}

recipe_r4_icache() {
# Round 4: instruction-cache and wait-state counters of the pipelined (config 2) and flattened (config 3)
# kernels: does instruction fetch explain the one-time phases' cycles?  One rocprofv3 pass per counter set
# (SQ issue/wait states + instruction fetch; SQC instruction-cache requests / hits / misses), each under
# its own kill timer.
for W in cfg3 cfg2; do
    timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH SQ_IFETCH_LEVEL \
        --kernel-trace --output-format csv -d gpurun_out/icache_sq_$W -o p -- \
        python3 bench.py --workload $W --steps 3 --warmup 1 --cpu-seconds 0 --no-graph --no-cold --forged 0 \
        > gpurun_out/icache_sq_$W.log 2>&1 || exit $?
    timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE \
        --kernel-trace --output-format csv -d gpurun_out/icache_sqc_$W -o p -- \
        python3 bench.py --workload $W --steps 3 --warmup 1 --cpu-seconds 0 --no-graph --no-cold --forged 0 \
        > gpurun_out/icache_sqc_$W.log 2>&1 || exit $?
done
python3 tools/pmc_summary.py gpurun_out/icache_sq_* gpurun_out/icache_sqc_* > gpurun_out/icache_summary.txt 2>&1
cat gpurun_out/icache_summary.txt
}

recipe_r4_last() {
# Round 4, last measurement on the final build: the default bench line with the host path, and the N = 4
# launcher path as the driver runs it with the four ranks sharing the GPU (RG_BENCH_SHARE_GPU=1).
timeout -k 10 400 python bench.py --e2e > gpurun_out/r4_last_default.jsonl 2> gpurun_out/r4_last_default.err && cat gpurun_out/r4_last_default.jsonl | cut -c1-600 &&
RG_BENCH_SHARE_GPU=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 4 --steps 5 --warmup 2 --cpu-seconds 2 > gpurun_out/r4_rehearse_torchrun4.jsonl 2> gpurun_out/r4_rehearse_torchrun4.err && cut -c1-400 gpurun_out/r4_rehearse_torchrun4.jsonl
}

recipe_r4_lb2() {
# Round 4, first look at real two-wave co-residency on config 2: the in-tree build against
# __launch_bounds__(256, 2) (tools/build_variant.sh lb2 -DRG_PIPE_LB2: the pipelined kernels forced
# into 256 VGPRs, so two 256-thread workgroups fit per CU), each with 1 and 2 lanes per packet.
run() { # name lib flags...
    local name=$1 lib=$2
    shift 2
    if [ "$lib" = base ]; then unset RG_AEAD_LIB; else export RG_AEAD_LIB=tools/build/librg_$lib.so; fi
    timeout -k 10 200 python bench.py --workload cfg2 --steps 20 --warmup 3 --cpu-seconds 0 --no-cold --forged 0 "$@" \
        >gpurun_out/r4lb2_$name.log 2>&1 || { echo "$name FAILED $?"; tail -5 gpurun_out/r4lb2_$name.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/r4lb2_$name.log') if l.startswith('{')][-1]); print('$name', d['value'], d['seal_ms'], d['open_ms'], d['config']['kernel'][:40])"
}
for rep in 1 2; do
    run base_l1_$rep base
    run lb2_l1_$rep lb2
    run base_l2w2_$rep base --lanes 2 --wg-per-cu 2
    run lb2_l2w2_$rep lb2 --lanes 2 --wg-per-cu 2
done
run base_l1_m1 base --debug-mode 1 --no-verify
run lb2_l2w2_m1 lb2 --lanes 2 --wg-per-cu 2 --debug-mode 1 --no-verify
run base_l2w2_m1 base --lanes 2 --wg-per-cu 2 --debug-mode 1 --no-verify
}

recipe_r4_mapped() {
# Round 4: the host path with descriptors, counters and statuses in mapped host memory (working tree)
# against the committed build (tools/build/librg_head.so, three copies per slice): host-path GPU tests,
# then tools/e2e_probe.py on configs 2 and 3 by slice size, interleaved.
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "host or group or sessions" --timeout 120 --timeout-method thread > gpurun_out/r4_mapped_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r4_mapped_tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
    for v in head base; do
        if [ "$v" = base ]; then unset RG_AEAD_LIB; else export RG_AEAD_LIB=tools/build/librg_$v.so; fi
        for w in cfg2 cfg3; do
            echo "== $v $w run $r"
            timeout -k 10 240 python tools/e2e_probe.py $w 4,8,16 || exit $?
        done
    done
done 2>&1 | tee gpurun_out/r4_e2e_mapped_ab.txt
}

recipe_r4_nobar() {
# Round 4: the flattened kernel without the workgroup barrier after the cut reads (one unit per wave: the
# shared slots are never written again): flat parity tests, then an interleaved A/B against the committed
# build on config 3.
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_forged.py -x -q -m gpu \
    -k "flat or open_failures or bad_descriptors or malformed or digest or auto" --timeout 300 --timeout-method thread \
    > gpurun_out/r4_nobar_tests.log 2>&1
rc=$?
tail -2 gpurun_out/r4_nobar_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/ab.sh "base head" "cfg3" 4 --no-cold --forged 0 2>&1 | tee gpurun_out/r4_cfg3_nobar_ab.txt
}

recipe_r4_pcie2() {
# Round 4: the bench line's e2e.pcie_ceiling with hipHostMalloc buffers (short bench run).
timeout -k 10 300 python bench.py --e2e --steps 5 --warmup 2 --cpu-seconds 0 --forged 0 --no-cold > gpurun_out/r4_pcie2.jsonl 2>gpurun_out/r4_pcie2.err && python3 -c "import json; d=json.loads(open('gpurun_out/r4_pcie2.jsonl').read()); print(d['e2e'])"
}

recipe_r4_perwave() {
# Round 4: the flattened kernel's slowest waves at config 3 -- each wave's first sub-unit (packets, chunks,
# steps) and XCD beside its phase cycles (diag build) -- and the GPU tests after the device-restore change.
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4_gputest2.log 2>&1
rc=$?
tail -2 gpurun_out/r4_gputest2.log
[ $rc -eq 0 ] || exit $rc
RG_AEAD_LIB=tools/build/librg_diag.so timeout -k 10 200 python tools/flat_stamps.py --workload cfg3 --per-wave > gpurun_out/r4_cfg3_perwave.txt 2>&1 && cat gpurun_out/r4_cfg3_perwave.txt
}

recipe_r4_perwave2() {
# Round 4, final build: the flattened kernel's per-wave phases on config 3 (diag build), after the carry
# power's top-bit change and the dropped barrier.
RG_AEAD_LIB=tools/build/librg_diag.so timeout -k 10 200 python tools/flat_stamps.py --workload cfg3 --per-wave > gpurun_out/r4_cfg3_perwave_final.txt 2>&1
rc=$?
head -3 gpurun_out/r4_cfg3_perwave_final.txt | cut -c1-600
exit $rc
}

recipe_r4_pieces() {
# Round 4: host path with downloads in 2 MiB pieces (working tree)
# against the committed build (tools/build/librg_head.so): host-path GPU tests, interleaved
# tools/e2e_probe.py on configs 2 and 3, then a copy + kernel trace of the working tree.
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "host or group or sessions or pinned" --timeout 120 --timeout-method thread > gpurun_out/r4_pieces_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r4_pieces_tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
    for v in head base; do
        if [ "$v" = base ]; then unset RG_AEAD_LIB; else export RG_AEAD_LIB=tools/build/librg_$v.so; fi
        for w in cfg2 cfg3; do
            echo "== $v $w run $r"
            timeout -k 10 240 python tools/e2e_probe.py $w 4,8,16 || exit $?
        done
    done
done 2>&1 | tee gpurun_out/r4_e2e_pieces_ab.txt
unset RG_AEAD_LIB
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/e2etrace7 -o run -- python3 tools/e2e_probe.py cfg2 8 > gpurun_out/e2etrace7.log 2>&1
}

recipe_r4_powtop() {
# Round 4: the flattened kernel with the carry power's top bit taken as a choice of 1 or r (one square-and-multiply step fewer):
# flat parity tests, then an interleaved A/B against the committed
# build on config 3.
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_forged.py -x -q -m gpu \
    -k "flat or open_failures or bad_descriptors or malformed or digest or auto" --timeout 300 --timeout-method thread \
    > gpurun_out/r4_powtop_tests.log 2>&1
rc=$?
tail -2 gpurun_out/r4_powtop_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/ab.sh "base head" "cfg3" 4 --no-cold --forged 0 2>&1 | tee gpurun_out/r4_cfg3_powtop_ab.txt
}

recipe_r4_profiles2() {
# Round 4, the profile set again on the final build (tile seal fast path, flat barrier dropped):
# default line, kernel stats, FETCH/WRITE passes, VALU counters, bench rows of every config.
bash tools/round_profiles.sh > gpurun_out/r4_profiles2.log 2>&1
rc=$?
tail -8 gpurun_out/r4_profiles2.log
exit $rc
}

recipe_r4_prologue() {
# Round 4: how many cycles the pipelined kernel spends before its first unit (kernel-argument loads, the
# walk's setup, the first descriptor): config 2 seal, one lane per packet, one workgroup per CU, stamps of
# the diag build (tools/coresidency.py reports the prologue beside the wave's cycles).
RG_AEAD_LIB=tools/build/librg_diag.so timeout -k 10 200 python tools/coresidency.py --workload cfg2 --lanes 1 --wg-per-cu 1 --mode 3 > gpurun_out/r4_pipe_prologue.json 2>gpurun_out/r4_pipe_prologue.err && cat gpurun_out/r4_pipe_prologue.json
}

recipe_r4_quadfuse() {
# Round 4: the first lane-quad key-block group fused with the one-lane pass (flattened kernel, phase A):
# flat / forged / malformed / digest GPU tests, interleaved A/B against the committed build on config 3,
# and the per-wave stamps by unit packet count (diag build).
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_forged.py -x -q -m gpu \
    -k "flat or open_failures or bad_descriptors or malformed or digest or auto" --timeout 300 --timeout-method thread \
    > gpurun_out/r4_quadfuse_tests.log 2>&1
rc=$?
tail -2 gpurun_out/r4_quadfuse_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/ab.sh "base head" "cfg3" 3 --no-cold --forged 0 &&
RG_AEAD_LIB=tools/build/librg_diag.so timeout -k 10 200 python tools/flat_stamps.py --workload cfg3 --per-wave > gpurun_out/r4_cfg3_perwave2.txt 2>&1 && grep -v "^slowest" gpurun_out/r4_cfg3_perwave2.txt
}

recipe_r4_search() {
# Round 4: where the flattened kernel's cooperative unit search spends its ~10 k cycles (diag build, search
# sub-stamps), and the ADVICE r3 regrow test of the MAC key table on a busy stream.
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "mac_verify" --timeout 120 --timeout-method thread > gpurun_out/r4_mac_tests.log 2>&1
rc=$?
tail -2 gpurun_out/r4_mac_tests.log
[ $rc -eq 0 ] || exit $rc
RG_AEAD_LIB=tools/build/librg_diag.so timeout -k 10 200 python tools/flat_stamps.py --workload cfg3 > gpurun_out/r4_cfg3_search_stamps.txt 2>&1 && cat gpurun_out/r4_cfg3_search_stamps.txt
}

recipe_r4_taper() {
# Round 4: the host-memory path with tapered slices (first and last a quarter of the span) and the small
# uploads moved off the frame stream: host-path GPU tests, then the slice-size probe for this build and the
# committed one (tools/build_rev.sh head) on the same box.
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "host or session or group or recv or send" --timeout 300 --timeout-method thread > gpurun_out/r4_taper_tests.log 2>&1
rc=$?
tail -2 gpurun_out/r4_taper_tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1; do
    timeout -k 10 300 python tools/e2e_probe.py cfg2 4,8,16,32 > gpurun_out/r4_taper_new_$r.jsonl && echo "new $r" && cat gpurun_out/r4_taper_new_$r.jsonl || exit 1
    RG_AEAD_LIB=tools/build/librg_head.so timeout -k 10 300 python tools/e2e_probe.py cfg2 16 > gpurun_out/r4_taper_head_$r.jsonl && echo "head $r" && cat gpurun_out/r4_taper_head_$r.jsonl || exit 1
done
}

recipe_r4_tilefull() {
# Round 4: the tile kernel's seal without Poly1305 predicates on chunks that are whole in every lane
# (c + 1 < the wave's smallest chunk count): the tile / digest / forged parity tests, then an interleaved
# A/B against the committed build on configs 4 and 5.
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_forged.py -x -q -m gpu \
    -k "tile or digest or random or large_payload or reference or openssl or cfg5 or forged or past_2" \
    --timeout 300 --timeout-method thread > gpurun_out/r4_tilefull_tests.log 2>&1
rc=$?
tail -2 gpurun_out/r4_tilefull_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/ab.sh "base head" "cfg4 cfg5" 3 --no-cold --forged 0 2>&1 | tee gpurun_out/r4_tilefull_ab.txt
}

recipe_r4_tilewhole() {
# Round 4: the tile kernel with a loop of its own for waves whose lanes all have the same chunk count (seal and open, no Poly1305 predicates before the last chunk)
# (c + 1 < the wave's smallest chunk count): the tile / digest / forged parity tests, then an interleaved
# A/B against the committed build on configs 4 and 5.
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_forged.py -x -q -m gpu \
    -k "tile or digest or random or large_payload or reference or openssl or cfg5 or forged or past_2" \
    --timeout 300 --timeout-method thread > gpurun_out/r4_tilewhole_tests.log 2>&1
rc=$?
tail -2 gpurun_out/r4_tilewhole_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/ab.sh "base head" "cfg4 cfg5" 3 --no-cold --forged 0 2>&1 | tee gpurun_out/r4_tilewhole_ab.txt
}

recipe_r4_weights() {
# Round 4: the cooperative search's work weights at config 3 -- a packet's one-time-key block counted as 1
# (base), 2 or 3 eighths of a chunk step (kCoopWPkt, variant builds wp2 / wp3) -- interleaved A/B.
bash tools/ab.sh "base wp2 wp3" "cfg3" 3 --no-cold --forged 0
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench_ranks.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4_bench_ranks_test.log 2>&1
rc=$?
tail -3 gpurun_out/r4_bench_ranks_test.log
exit $rc
}

recipe_r4_wholegroups() {
# Round 4: the flattened kernel's whole-group unit rule (> 1024 packets per unit) against the oracle.
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu -k "whole_groups" --timeout 400 --timeout-method thread > gpurun_out/r4_wholegroups.log 2>&1
rc=$?
tail -3 gpurun_out/r4_wholegroups.log
exit $rc
}

recipe_r5_a() {
# Round 5: every GPU test on the stream-ordered-wipe build, then the one-process group line rehearsed with
# two contexts on one GPU (device-resident config 5 split + the e2e_multi host-memory leg).
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash tools/gpu_run.sh test && \
RG_BENCH_SHARE_GPU=1 timeout -k 10 400 python bench.py --single-process --gpus 2 --steps 5 --warmup 2 > gpurun_out/sp2.log 2>&1; echo rc=$?; tail -c 3000 gpurun_out/sp2.log
}

recipe_r5_e2eenv() {
# Round 5: which engine carries the host path's download.  tools/e2e_probe.py (cfg2,
# 8 MiB slices) under runtime settings that may move the D2H copy off the shader blit kernel, each with a
# kernel + memory-copy trace (a D2H memory-copy record = SDMA, a __amd_rocclr_copyBuffer kernel = blit).
mkdir -p gpurun_out/e2eenv
for cfg in base GPU_FORCE_BLIT_COPY_SIZE=0 DEBUG_CLR_LIMIT_BLIT_WG=16 DEBUG_CLR_LIMIT_BLIT_WG=64 GPU_CP_DMA_COPY_SIZE=0; do
    echo "== $cfg"
    if [ "$cfg" = base ]; then envs=(X_RG_NONE=1); else envs=("$cfg"); fi
    env "${envs[@]}" timeout -k 10 120 python3 tools/e2e_probe.py cfg2 8 > "gpurun_out/e2eenv/$cfg.log" 2>&1 || { echo "rc=$?"; tail -5 "gpurun_out/e2eenv/$cfg.log"; return 1; }
    tail -1 "gpurun_out/e2eenv/$cfg.log"
    env "${envs[@]}" timeout -k 10 150 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "gpurun_out/e2eenv/tr_$cfg" -o run -- python3 tools/e2e_probe.py cfg2 8 > "gpurun_out/e2eenv/tr_$cfg.log" 2>&1 || { echo "trace rc=$?"; return 1; }
    python3 tools/e2e_timeline.py "gpurun_out/e2eenv/tr_$cfg" seal 2>&1 | tail -14
done
}

recipe_refresh_tiles() {
# refresh after the dynamic tile deal: default line, bench rows, cfg4 stats, cfg4/cfg5 traffic
G="bash tools/gpu_run.sh"
$G default || exit $?
RG_WORKLOAD=cfg4 $G prof || exit $?
for W in cfg4 cfg5; do RG_WORKLOAD=$W $G pmc_hbm || exit $?; done
RG_WORKLOADS="cfg4" $G valu || exit $?
RG_WORKLOADS="cfg2 cfg3 cfg4 cfg5" $G bench_all || exit $?
}

recipe_tile_dyn() {
# tile kernel dynamic deal: GPU tests, A/B against the static deal on cfg4/cfg5, stamps
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/dyn_pytest.log 2>&1; rc=$?; tail -n 3 gpurun_out/dyn_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 bash tools/ab.sh "base dyn0" "cfg4 cfg5" 2 --no-cold || exit $?
timeout -k 10 200 python tools/stamps.py --workload cfg4 > gpurun_out/cfg4_stamps_dyn.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/cfg4_stamps_dyn.log | python3 -c "
import sys,json; d=json.loads(sys.stdin.read())
for k,v in d.items(): print(k, v['wave_us_pct_0_10_50_90_99_100'], v['shader_clock_ghz'], v['share'])"
}

recipe_tile_fair() {
# tile kernel fair SIMD issue (s_setprio by progress): tile-path GPU tests, A/B on cfg4/cfg5, stamps
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/fair_pytest.log 2>&1; rc=$?; tail -n 3 gpurun_out/fair_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 bash tools/ab.sh "base fair0 dyn0" "cfg4 cfg5" 2 --no-cold || exit $?
timeout -k 10 200 python tools/stamps.py --workload cfg4 > gpurun_out/cfg4_stamps_fair.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/cfg4_stamps_fair.log | python3 -c "
import sys,json; d=json.loads(sys.stdin.read())
for k,v in d.items(): print(k, v['wave_us_pct_0_10_50_90_99_100'], v['shader_clock_ghz'], v['share'])"
}

recipe_tile_pool() {
# tile kernel global tail pool: GPU tests, A/B on cfg4/cfg5, stamps
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pool_pytest.log 2>&1; rc=$?; tail -n 3 gpurun_out/pool_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 bash tools/ab.sh "base pool0" "cfg4 cfg5" 3 --no-cold || exit $?
timeout -k 10 200 python tools/stamps.py --workload cfg4 > gpurun_out/cfg4_stamps_pool.log 2>&1 || exit $?
python3 - <<'PY'
import numpy as np
for op in ('seal','open'):
    d=np.load(f'gpurun_out/stamps_raw_cfg4_{op}.npy')[:2048]
    rt=d[:,7]/100.0; wg=rt.reshape(256,8)
    print(op,'dur pct', np.percentile(rt,[0,10,50,90,100]).round(1), 'per-CU max pct', np.percentile(wg.max(1),[0,50,100]).round(1))
PY
}

recipe_tile_pool2() {
# tile pool prefetch: tests on the pool-from-2-rounds build, A/B base (pool from 16 rounds, ahead) / pmin2 / pmin2noahead
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
RG_AEAD_LIB=tools/build/librg_pmin2.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "tile_dynamic_deal or digest or tile_g2" --timeout 120 --timeout-method thread > gpurun_out/pool2_pytest.log 2>&1; rc=$?; tail -n 2 gpurun_out/pool2_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 bash tools/ab.sh "base pmin2 pmin2noahead" "cfg4 cfg5" 3 --no-cold || exit $?
}

recipe_ab_lib() {
# A/B of variant libraries (tools/build/librg_<name>.so; "base" = the in-tree library) on one workload,
# alternating, two rounds:  LIBS="base w8" W=cfg3 FLAGS="--staged 3" tools/recipes.sh ab_lib
for rep in 1 2; do
    for v in ${LIBS:-base}; do
        if [ $v = base ]; then L=""; else L="RG_AEAD_LIB=tools/build/librg_$v.so"; fi
        env $L timeout -k 10 200 python bench.py --workload ${W:-cfg3} ${FLAGS:-} --steps 20 --warmup 3 --cpu-seconds 0 --no-cold > gpurun_out/ab_${v}_$rep.log 2>&1 || exit 1
        python3 -c "import json; d=json.loads([l for l in open('gpurun_out/ab_${v}_$rep.log') if l.startswith('{')][-1]); print('$v', $rep, d['value'], d['seal_ms'], d['open_ms'])"
    done
done
}

recipe_ab_tile() {
set -e
for rep in 1 2; do
for v in new old; do
  for sh in 0 112; do
    if [ $v = old ]; then L="RG_AEAD_LIB=tools/build/librg_oldtile.so"; else L=""; fi
    env $L timeout -k 10 200 python bench.py --workload cfg4 --frame-shift $sh --steps 20 --warmup 3 --cpu-seconds 0 --no-cold > gpurun_out/ab_${v}_${sh}_$rep.log 2>&1
    python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/ab_${v}_${sh}_$rep.log') if l.startswith('{')][-1]); print('$v', $sh, $rep, d['value'], d['seal_ms'], d['open_ms'])"
  done
done
done
}

recipe_abl_flat() {
# flat-kernel phase stamps under diagnostic ablation builds (tools/build/librg_<name>.so)
for v in base ${ABL:-nostore noload nopoly nomem}; do
    if [ $v = base ]; then L=""; else L="RG_AEAD_LIB=tools/build/librg_$v.so"; fi
    echo "== $v"
    env $L timeout -k 10 120 python tools/flat_stamps.py --workload ${W:-cfg3} --plan 1 | grep '^seal' || exit 1
done
}

recipe_r3_check() {
# round-3 check: forged-frame tests, parity suite, default bench line, forged bench (one GPU call)
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step() { # name timeout cmd...
    local name=$1 to=$2; shift 2
    echo "== $name $(date +%T)"
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "rc=$rc"; tail -n 4 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop after $name"; exit $rc; fi
}
for s in "$@"; do
    case $s in
    forged) step forged 600 python -u -m pytest tests/test_gpu_forged.py -x -v --timeout 120 --timeout-method thread ;;
    parity) step parity 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sessions.py tests/test_gpu_sessions_dev.py -v --timeout 120 --timeout-method thread ;;
    allgpu) step allgpu 1000 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread ;;
    bench) step bench 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 ;;
    bench_forged) step bench_forged 300 python bench.py --steps 10 --warmup 3 --no-cold --cpu-seconds 0 --forged 0.1 ;;
    bench_forged1) step bench_forged1 300 python bench.py --steps 10 --warmup 3 --no-cold --cpu-seconds 0 --forged 0.01 ;;
    bench_cfg4f) step bench_cfg4f 300 python bench.py --workload cfg4 --steps 5 --warmup 2 --no-cold --cpu-seconds 0 --forged 0.1 ;;
    bench_all) for w in cfg2 cfg3 cfg4 cfg5; do step bench_$w 300 python bench.py --workload $w --steps 10 --warmup 3 --no-cold --cpu-seconds 0; done ;;
    prof) step prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cold --cpu-seconds 0 ;;
    esac
done
}

recipe_round3_profiles_a() {
# round 3 final profiles, part A: default bench line, rocprofv3 kernel stats per config, bench rows of every config
G="bash tools/gpu_run.sh"
$G default || exit $?
for W in cfg2 cfg3 cfg4; do RG_WORKLOAD=$W $G prof || exit $?; done
RG_WORKLOADS="cfg2 cfg3 cfg4 cfg5" $G bench_all || exit $?
echo "round profiles A done"
}

recipe_round3_profiles_b() {
# round 3 final profiles, part B: FETCH_SIZE / WRITE_SIZE passes per config and the VALU issue counters
G="bash tools/gpu_run.sh"
for W in cfg2 cfg3 cfg4 cfg5; do RG_WORKLOAD=$W $G pmc_hbm || exit $?; done
RG_WORKLOADS="cfg2 cfg3 cfg4" $G valu || exit $?
echo "round profiles B done"
}

recipe_r5_hostpoll() {
# Round 5: the host path's chain.  The round-4 HIP API trace shows every slice's kernel
# and download reaching the GPU only at the host thread's next HIP call after a blocking hipEventSynchronize
# (deferred submission of commands behind a cross-stream event).  A/B: the thread polls hipEventQuery
# instead of blocking (tools/build/librg_poll.so, -DRG_HOST_POLL=1) against the in-tree build, interleaved,
# then a kernel + copy + HIP API trace of the poll build.
mkdir -p gpurun_out/hostpoll
for rep in 1 2; do
    for lib in base poll; do
        if [ $lib = base ]; then L=(X_RG_NONE=1); else L=(RG_AEAD_LIB=tools/build/librg_$lib.so); fi
        env "${L[@]}" timeout -k 10 120 python3 tools/e2e_probe.py cfg2 4,8,16 > gpurun_out/hostpoll/${lib}_$rep.jsonl 2>&1 || { echo "rc=$?"; tail -3 gpurun_out/hostpoll/${lib}_$rep.jsonl; return 1; }
        echo "== $lib $rep"; cat gpurun_out/hostpoll/${lib}_$rep.jsonl
    done
done
RG_AEAD_LIB=tools/build/librg_poll.so timeout -k 10 150 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/hostpoll/tr -o run -- python3 tools/e2e_probe.py cfg2 8 > gpurun_out/hostpoll/tr.log 2>&1 || { echo "trace rc=$?"; return 1; }
python3 tools/e2e_timeline.py gpurun_out/hostpoll/tr seal 2>&1 | tail -16
}

recipe_r5_hostup() {
# Round 5: the host path's upload chain.  Polling instead of a blocking wait changed nothing
# (r5_hostpoll): consecutive 8 MiB uploads on one stream leave ~33 us gaps, and each slice's kernel
# starts with the NEXT upload, ~35 us after its own upload ended.  A/B of one upload stream per slot
# (up1) and of the kernel in its upload's stream as well (up2) against the in-tree build, interleaved,
# with a trace of each variant.
mkdir -p gpurun_out/hostup
for rep in 1 2; do
    for lib in base up1 up2; do
        if [ $lib = base ]; then L=(X_RG_NONE=1); else L=(RG_AEAD_LIB=tools/build/librg_$lib.so); fi
        env "${L[@]}" timeout -k 10 120 python3 tools/e2e_probe.py cfg2 4,8,16 > gpurun_out/hostup/${lib}_$rep.jsonl 2>&1 || { echo "rc=$?"; tail -3 gpurun_out/hostup/${lib}_$rep.jsonl; return 1; }
        echo "== $lib $rep"; grep slice gpurun_out/hostup/${lib}_$rep.jsonl
    done
done
for lib in up1 up2; do
    RG_AEAD_LIB=tools/build/librg_$lib.so timeout -k 10 150 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/hostup/tr_$lib -o run -- python3 tools/e2e_probe.py cfg2 8 > gpurun_out/hostup/tr_$lib.log 2>&1 || { echo "trace rc=$?"; return 1; }
    echo "== trace $lib"; python3 tools/e2e_timeline.py gpurun_out/hostup/tr_$lib seal 2>&1 | tail -14
done
}

recipe_r5_hostslots() {
# Round 5: per-slot upload streams moved nothing (r5_hostup): in their trace each upload starts ~35 us
# after the download three slices back ends -- the slot it reuses.  A/B of 4 and 6 slots (s4, s6) and of 6
# slots with one upload stream each (s6up) against the in-tree 3-slot build, then a trace of s6.
mkdir -p gpurun_out/hostslots
for rep in 1 2; do
    for lib in base s4 s6 s6up; do
        if [ $lib = base ]; then L=(X_RG_NONE=1); else L=(RG_AEAD_LIB=tools/build/librg_$lib.so); fi
        env "${L[@]}" timeout -k 10 120 python3 tools/e2e_probe.py cfg2 2,4,8,16 > gpurun_out/hostslots/${lib}_$rep.jsonl 2>&1 || { echo "rc=$?"; tail -3 gpurun_out/hostslots/${lib}_$rep.jsonl; return 1; }
        echo "== $lib $rep"; grep slice gpurun_out/hostslots/${lib}_$rep.jsonl
    done
done
RG_AEAD_LIB=tools/build/librg_s6.so timeout -k 10 150 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/hostslots/tr_s6 -o run -- python3 tools/e2e_probe.py cfg2 8 > gpurun_out/hostslots/tr_s6.log 2>&1 || { echo "trace rc=$?"; return 1; }
python3 tools/e2e_timeline.py gpurun_out/hostslots/tr_s6 seal 2>&1 | tail -14
}

recipe_r5_hostalloc() {
# Round 5: more slots made the host path slower, and a trace of six slots shows each slice's kernel and
# the next upload released only when the previous download (a __amd_rocclr_copyBuffer shader blit) ends.
# Does the caller's host allocation decide the download's engine?  tools/e2e_probe.py with the frames in
# hipHostMalloc buffers of other flags (coherent, non-coherent, mapped+portable, write-combined; variant
# libraries' rg_host_alloc) against the default, then a trace of each.
mkdir -p gpurun_out/hostalloc
for lib in base hcoh hnc hmap hwc; do
    if [ $lib = base ]; then L=(X_RG_NONE=1); else L=(RG_AEAD_LIB=tools/build/librg_$lib.so); fi
    env "${L[@]}" timeout -k 10 120 python3 tools/e2e_probe.py cfg2 8,16 > gpurun_out/hostalloc/$lib.jsonl 2>&1 || { echo "rc=$?"; tail -3 gpurun_out/hostalloc/$lib.jsonl; return 1; }
    echo "== $lib"; grep slice gpurun_out/hostalloc/$lib.jsonl
    env "${L[@]}" timeout -k 10 150 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/hostalloc/tr_$lib -o run -- python3 tools/e2e_probe.py cfg2 8 > gpurun_out/hostalloc/tr_$lib.log 2>&1 || { echo "trace rc=$?"; return 1; }
    python3 tools/e2e_timeline.py gpurun_out/hostalloc/tr_$lib seal 2>&1 | tail -7
done
}

recipe_r5_hostev() {
# Round 5: in the round-4 API trace the host's wait for slot k-3's download event returns only when the
# download of slice k-2 ends: the event recorded behind a download seems to complete with the NEXT
# packet of that stream, so the three-slot pipeline runs two deep.  A/B: events with timing (ev1), a
# hipStreamQuery of the download stream after each record (ev2), an empty kernel behind each record
# (ev3), against the in-tree build, interleaved; then the HIP API + kernel + copy trace of each.
mkdir -p gpurun_out/hostev
for rep in 1 2; do
    for lib in base ev1 ev2 ev3; do
        if [ $lib = base ]; then L=(X_RG_NONE=1); else L=(RG_AEAD_LIB=tools/build/librg_$lib.so); fi
        env "${L[@]}" timeout -k 10 120 python3 tools/e2e_probe.py cfg2 4,8,16 > gpurun_out/hostev/${lib}_$rep.jsonl 2>&1 || { echo "rc=$?"; tail -3 gpurun_out/hostev/${lib}_$rep.jsonl; return 1; }
        echo "== $lib $rep"; grep slice gpurun_out/hostev/${lib}_$rep.jsonl
    done
done
for lib in ev1 ev3; do
    RG_AEAD_LIB=tools/build/librg_$lib.so timeout -k 10 150 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/hostev/tr_$lib -o run -- python3 tools/e2e_probe.py cfg2 8 > gpurun_out/hostev/tr_$lib.log 2>&1 || { echo "trace rc=$?"; return 1; }
    echo "== trace $lib"; python3 tools/e2e_timeline.py gpurun_out/hostev/tr_$lib seal 2>&1 | tail -8
done
}

recipe_r5_deal() {
# Round 5: the flattened kernel's units dealt in size order, snake-wise (every unit 4096 / kgc packets; config
# 3: 64) instead of contiguous cuts: flat / forged / digest / coop GPU tests, interleaved A/B against the
# committed build (tools/build_rev.sh head) on config 3, per-wave phases of the diag build, the splitbench
# two-chain Poly1305 variants.
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_forged.py -x -q -m gpu \
    -k "flat or open_failures or bad_descriptors or malformed or digest or auto or coop" --timeout 300 --timeout-method thread \
    > gpurun_out/r5_deal_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r5_deal_tests.log
[ $rc -eq 0 ] || return $rc
bash tools/ab.sh "base head" "cfg3" 3 --no-cold --forged 0 || return $?
RG_AEAD_LIB=tools/build/librg_diag.so timeout -k 10 200 python tools/flat_stamps.py --workload cfg3 --per-wave > gpurun_out/r5_cfg3_perwave.txt 2>&1 && tail -6 gpurun_out/r5_cfg3_perwave.txt | cut -c1-1500 || return $?
[ -n "${R5_SPLIT:-}" ] && { timeout -k 10 60 tools/build/splitbench > gpurun_out/r5_splitbench.json && cat gpurun_out/r5_splitbench.json; }
[ -n "${R5_PMC:-}" ] && { RG_WORKLOAD=cfg3 bash tools/gpu_run.sh pmc_hbm || return $?; }
return 0
}

recipe_r5_check() {
# Round 5: every GPU test on the current build, smoke(), the default bench line as the driver runs it, and
# the N = 2 launcher path rehearsed on one GPU (torch.distributed.run, two ranks sharing the GPU over gloo;
# its line now carries e2e_multi).
bash tools/gpu_run.sh test smoke || return $?
timeout -k 10 600 python bench.py > gpurun_out/r5_default.jsonl 2> gpurun_out/r5_default.err || { tail -5 gpurun_out/r5_default.err; return 1; }
cut -c1-600 gpurun_out/r5_default.jsonl
RG_BENCH_SHARE_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 5 --warmup 2 --cpu-seconds 2 \
    > gpurun_out/r5_rehearse_tr2.log 2>&1
rc=$?; grep '^{' gpurun_out/r5_rehearse_tr2.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d.get('speedup'), json.dumps(d.get('e2e_multi'))[:800])"
[ $rc -ne 0 ] && { tail -20 gpurun_out/r5_rehearse_tr2.log; return $rc; }
return 0
}

recipe_r5_sw() {
# Round 5: store waves for the pipelined kernel's line stores (RG_STORE_WAVE builds: a partner wave per
# SIMD reads the ring back and stores): every GPU test on that build, per-wave stamps of the diag builds
# with and without, and the SQ issue counters of both on config 2.
if [ -z "${R5_NOTEST:-}" ]; then
    RG_AEAD_LIB=tools/build/librg_${R5_SW:-sw}.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 \
        --timeout-method thread > gpurun_out/r5_sw_tests.log 2>&1
    rc=$?; tail -2 gpurun_out/r5_sw_tests.log; [ $rc -eq 0 ] || return $rc
fi
for v in dg dgsw; do
    RG_AEAD_LIB=tools/build/librg_$v.so timeout -k 10 200 python tools/stamps.py --workload cfg2 > gpurun_out/r5_sw_st_$v.log 2>&1 \
        || { tail -5 gpurun_out/r5_sw_st_$v.log; return 1; }
    tail -4 gpurun_out/r5_sw_st_$v.log | cut -c1-600
done
for v in base ${R5_SW:-sw}; do
    if [ $v = base ]; then unset RG_AEAD_LIB; else export RG_AEAD_LIB=tools/build/librg_$v.so; fi
    timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAVES SQ_ACTIVE_INST_VALU \
        SQ_WAIT_ANY SQ_WAIT_INST_ANY --kernel-trace --output-format csv -d gpurun_out/r5_sw_pmc_$v -o p -- \
        python3 bench.py --workload cfg2 --steps 5 --warmup 2 --cpu-seconds 0 --no-graph > gpurun_out/r5_sw_pmc_$v.log 2>&1 || return $?
done
unset RG_AEAD_LIB
python3 tools/pmc_clock.py gpurun_out/r5_sw_pmc_* 2>&1 | tail -12
return 0
}

recipe_r5_cut() {
# Round 5: the flattened kernel's cut points, each wave its own two from a workgroup-shared prefix (one
# barrier instead of two, no wave computing the others' cuts): flat / forged / digest / coop GPU tests on the
# variant, interleaved A/B on config 3, per-wave phases of both diag builds.
V=${R5_CUT:-cut2}
RG_AEAD_LIB=tools/build/librg_$V.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_forged.py -x -q \
    -m gpu -k "flat or open_failures or bad_descriptors or malformed or digest or auto or coop" --timeout 300 \
    --timeout-method thread > gpurun_out/r5_cut_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5_cut_tests.log; [ $rc -eq 0 ] || return $rc
bash tools/ab.sh "base ${R5_CUT_AB:-$V}" "cfg3" 3 --no-cold --forged 0 || return $?
for v in ${R5_CUT_ST:-diag ${V}dg}; do
    RG_AEAD_LIB=tools/build/librg_$v.so timeout -k 10 200 python tools/flat_stamps.py --workload cfg3 > gpurun_out/r5_cut_st_$v.txt 2>&1 \
        || { tail -5 gpurun_out/r5_cut_st_$v.txt; return 1; }
    grep -E "^(seal|open)" gpurun_out/r5_cut_st_$v.txt | cut -c1-900
done
return 0
}

recipe_r5_gthr() {
# Round 5: a group's host calls with one worker thread per context (RG_GROUP_THREADS, default on) against the
# single-thread loop (tools/build_variant.sh gthr0 -DRG_GROUP_THREADS=0): every GPU test and smoke() on the
# in-tree build first, config 3's profiles for the one-barrier search, then the --single-process line with
# 2 and 4 contexts sharing the one GPU (e2e_multi).
bash tools/gpu_run.sh test smoke || return $?
RG_WORKLOAD=cfg3 bash tools/gpu_run.sh prof pmc_hbm || return $?
RG_WORKLOADS=cfg3 bash tools/gpu_run.sh valu bench_all || return $?
for v in base gthr0; do
    for n in 2 4; do
        if [ $v = base ]; then unset RG_AEAD_LIB; else export RG_AEAD_LIB=tools/build/librg_$v.so; fi
        RG_BENCH_SHARE_GPU=1 timeout -k 10 400 python bench.py --single-process --gpus $n --steps 5 --warmup 2 \
            --cpu-seconds 0 > gpurun_out/r5_gthr_${v}_$n.log 2>&1 || return $?
        grep '^{' gpurun_out/r5_gthr_${v}_$n.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$v', $n, json.dumps(d.get('e2e_multi'))[:700])"
    done
done
unset RG_AEAD_LIB
return 0
}

recipe_r5_seg() {
# Round 5: the flattened kernel's stores in whole 64-byte segments (a chunk's pieces whose segment the next chunk
# completes held one step; a seal's DataHeader stored with the packet's first chunk): flat / forged / digest /
# coop / auto / malformed GPU tests on the variant (tools/build_variant.sh seg) and the group tests on the in-tree
# build, interleaved A/B on config 3, FETCH / WRITE passes of the variant (gpurun_out/pmc_*_cfg3).
RG_AEAD_LIB=tools/build/librg_seg.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_forged.py -x -q \
    -m gpu -k "flat or open_failures or bad_descriptors or malformed or digest or auto or coop" --timeout 300 \
    --timeout-method thread > gpurun_out/r5_seg_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5_seg_tests.log; [ $rc -eq 0 ] || return $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_group.py -x -q -m gpu --timeout 300 --timeout-method thread \
    > gpurun_out/r5_group_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5_group_tests.log; [ $rc -eq 0 ] || return $rc
bash tools/ab.sh "base seg" "cfg3" 3 --no-cold --forged 0 || return $?
RG_AEAD_LIB=tools/build/librg_seg.so RG_WORKLOAD=cfg3 bash tools/gpu_run.sh pmc_hbm > /dev/null || return $?
python3 tools/make_profiles.py --tag r5seg --workload cfg3 --fetch gpurun_out/pmc_fetch_cfg3 --write gpurun_out/pmc_write_cfg3 \
    --bench gpurun_out/ab_seg_cfg3_1.log 2>&1 | tail -12
return 0
}

recipe_r5_nosdma() {
# Round 5: the host path with every copy on a shader blit kernel (HSA_ENABLE_SDMA=0: no SDMA engine, so no
# cross-engine completion in the slice chain) against the default (SDMA uploads, blit downloads):
# tools/e2e_probe.py cfg2 at 4 / 8 / 16 MiB slices, interleaved, then a kernel + memory-copy trace of each.
mkdir -p gpurun_out/nosdma
for rep in 1 2; do
    for cfg in base HSA_ENABLE_SDMA=0; do
        if [ "$cfg" = base ]; then envs=(X_RG_NONE=1); else envs=("$cfg"); fi
        env "${envs[@]}" timeout -k 10 200 python3 tools/e2e_probe.py cfg2 4,8,16 > "gpurun_out/nosdma/${cfg}_$rep.log" 2>&1 \
            || { echo "rc=$?"; tail -5 "gpurun_out/nosdma/${cfg}_$rep.log"; return 1; }
        echo "$cfg $rep: $(tail -3 gpurun_out/nosdma/${cfg}_$rep.log | tr '\n' ' ')"
    done
done
for cfg in base HSA_ENABLE_SDMA=0; do
    if [ "$cfg" = base ]; then envs=(X_RG_NONE=1); else envs=("$cfg"); fi
    env "${envs[@]}" timeout -k 10 150 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "gpurun_out/nosdma/tr_$cfg" \
        -o run -- python3 tools/e2e_probe.py cfg2 8 > "gpurun_out/nosdma/tr_$cfg.log" 2>&1 || { echo "trace rc=$?"; return 1; }
    python3 tools/e2e_timeline.py "gpurun_out/nosdma/tr_$cfg" seal 2>&1 | tail -16
done
return 0
}

recipe_r5_pmcst() {
# Round 5: where config 2's store cost goes -- memory-pipe issue and stall counters of the pipelined seal
# with payload stores (mode 0), without them (mode 7) and compute only (mode 1), diag build, two --pmc passes
# each (8 SQ; 2 SQ + 2 TA + 3 TCP), summarised per wave by tools/valu_profile.py's reader.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || return 1
mkdir -p gpurun_out/pmcst
local P1="SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_ANY SQ_WAVES GRBM_GUI_ACTIVE"
local P2="SQ_WAVE_CYCLES SQ_WAVES TA_DATA_STALLED_BY_TC_CYCLES TA_ADDR_STALLED_BY_TC_CYCLES TCP_PENDING_STALL_CYCLES TCP_LFIFO_STALL_CYCLES TCP_RFIFO_STALL_CYCLES GRBM_GUI_ACTIVE"
local mode pass C extra
for mode in 0 7 1; do
    extra=""; [ $mode != 0 ] && extra="--debug-mode $mode --no-verify"
    for pass in 1 2; do
        if [ $pass = 1 ]; then C=$P1; else C=$P2; fi
        RG_AEAD_LIB=tools/build/librg_diag.so timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv \
            -d gpurun_out/pmcst/m${mode}_p$pass -o p -- python3 bench.py --workload cfg2 --steps 5 --warmup 2 \
            --cpu-seconds 0 --no-cold --no-graph --forged 0 $extra > gpurun_out/pmcst/m${mode}_p$pass.log 2>&1 \
            || { echo "fail mode $mode pass $pass"; tail -5 gpurun_out/pmcst/m${mode}_p$pass.log; return 1; }
    done
done
python3 - <<'PY'
import sys
sys.path.insert(0, "tools")
from valu_profile import summarise
for mode in (0, 7, 1):
    for p in (1, 2):
        for k, v in summarise(f"gpurun_out/pmcst/m{mode}_p{p}").items():
            if "seal" not in k:
                continue
            w = max(v["raw_means"].get("SQ_WAVES", 1), 1)
            per = {c: round(x / w) for c, x in v["raw_means"].items() if c not in ("SQ_WAVES", "GRBM_GUI_ACTIVE")}
            print(f"mode {mode} pass {p} {k.split('(')[0][-28:]} dur={v['duration_us_median']}us per-wave {per}")
PY
}

recipe_r5_rtenv() {
# Round 5: runtime signal settings against the host path's ~33 us completion chain (end-to-end):
# interrupts off (busy-polled signals) and an active-wait window; tools/e2e_probe.py cfg2
# at 8 / 16 MiB slices, interleaved with the default, two rounds.
mkdir -p gpurun_out/rtenv
local rep cfg
for rep in 1 2; do
    for cfg in X_RG_NONE=1 HSA_ENABLE_INTERRUPT=0 ROC_ACTIVE_WAIT_TIMEOUT=200; do  # (ROC_SYSTEM_SCOPE_SIGNAL=0 hangs)
        env "$cfg" timeout -k 10 200 python3 tools/e2e_probe.py cfg2 8,16 > "gpurun_out/rtenv/${cfg}_$rep.log" 2>&1 \
            || { echo "rc=$? $cfg"; tail -5 "gpurun_out/rtenv/${cfg}_$rep.log"; return 1; }
        echo "$cfg $rep: $(grep '^{' gpurun_out/rtenv/${cfg}_$rep.log | tr '\n' ' ')"
    done
done
return 0
}

recipe_r5_sched() {
# Round 5: LLVM's machine scheduler strategy. iterative-ilp fills most hazard s_nops with independent
# instructions (pipelined seal 604 -> 159 s_nop, flattened 425 -> 135, tile 893 -> 383) but spills in the
# G = 2 tile kernel. Builds: tools/build_variant.sh iilp -mllvm -amdgpu-sched-strategy=iterative-ilp (all
# kernels), VAR_ONLY="rg_pipe.hip rg_flat.hip" ... iilppf (pipelined and flattened only), ilp (max-ilp).
# Parity on iilp (the whole GPU suite), then an interleaved A/B.
cd "$GRAFT_REPO_ROOT" || return 1
RG_AEAD_LIB=tools/build/librg_iilp.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/sched_tests.log 2>&1 || { echo "tests rc=$?"; tail -20 gpurun_out/sched_tests.log; return 1; }
tail -2 gpurun_out/sched_tests.log
bash tools/ab.sh "${R5_SCHED_LIBS:-base iilp iilppf}" "${R5_SCHED_WS:-cfg2 cfg3 cfg4}" "${R5_SCHED_REPS:-2}"
}

recipe_r5_sched2() {
# Round 5: the kept build (iterative-ilp for the pipelined and flattened kernels, rustyguard_amd/build.py
# FILE_FLAGS) against the commit before it (tools/build_rev.sh old, built from that commit:
# default scheduler), three interleaved rounds on configs 2 and 3, then the GPU suite on the kept build and
# a rocprofv3 kernel-trace of the default command.
cd "$GRAFT_REPO_ROOT" || return 1
bash tools/ab.sh "base old" "cfg2 cfg3" 3 || return 1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/sched2_tests.log 2>&1 || { echo "tests rc=$?"; tail -20 gpurun_out/sched2_tests.log; return 1; }
tail -1 gpurun_out/sched2_tests.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || return 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sched2_prof -o run \
    -- python3 bench.py > gpurun_out/sched2_default.jsonl 2> gpurun_out/sched2_default.err || { echo "prof rc=$?"; return 1; }
grep -h "seal_kernel\|open_kernel" $(find gpurun_out/sched2_prof -name "*kernel_stats.csv") | cut -c1-160
}

recipe_r5_stamps_ilp() {
# Round 5: per-wave stamps on the kept build (ILP schedule; diag build with the same flags): the pipelined
# kernel's wave cycles at config 2 (seal mode 3, and compute-only mode 1), the flattened kernel's phases at
# config 3.
cd "$GRAFT_REPO_ROOT" || return 1
export RG_AEAD_LIB=tools/build/librg_diag.so
timeout -k 10 200 python tools/stamps.py --workload cfg2 > gpurun_out/r5_stamps_cfg2_ilp.txt 2>&1 || { tail -5 gpurun_out/r5_stamps_cfg2_ilp.txt; return 1; }
timeout -k 10 200 python tools/stamps.py --workload cfg2 --mode 1 > gpurun_out/r5_stamps_cfg2_m1_ilp.txt 2>&1 || { tail -5 gpurun_out/r5_stamps_cfg2_m1_ilp.txt; return 1; }
timeout -k 10 200 python tools/flat_stamps.py --workload cfg3 > gpurun_out/r5_flat_stamps_ilp.txt 2>&1 || { tail -5 gpurun_out/r5_flat_stamps_ilp.txt; return 1; }
grep -v "^/opt" gpurun_out/r5_stamps_cfg2_ilp.txt gpurun_out/r5_stamps_cfg2_m1_ilp.txt gpurun_out/r5_flat_stamps_ilp.txt | cut -c1-220
}

recipe_r5_dlen() {
# Round 5: the cooperative search's 16 length loads as buffer loads with a scalar offset per row (no 64-bit
# address arithmetic before them) against the commit before (tools/build_rev.sh prev): flat/coop/forged/
# digest GPU tests on the working tree, three interleaved config-3 rounds, then stamps of the phases.
cd "$GRAFT_REPO_ROOT" || return 1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "flat or coop or forged or digest or imix or random" \
    > gpurun_out/dlen_tests.log 2>&1 || { echo "tests rc=$?"; tail -20 gpurun_out/dlen_tests.log; return 1; }
tail -1 gpurun_out/dlen_tests.log
bash tools/ab.sh "base prev" "cfg3" 3 || return 1
RG_AEAD_LIB=tools/build/librg_diag.so timeout -k 10 200 python tools/flat_stamps.py --workload cfg3 > gpurun_out/r5_flat_stamps_dlen.txt 2>&1 \
    || { tail -5 gpurun_out/r5_flat_stamps_dlen.txt; return 1; }
grep -v "^/opt" gpurun_out/r5_flat_stamps_dlen.txt | cut -c1-700
}

recipe_r5_tile_sched() {
# Round 5: the tile kernel under iterative-maxocc (VAR_ONLY="rg_tile.hip" tools/build_variant.sh tmaxocc
# -mllvm -amdgpu-sched-strategy=iterative-maxocc): the G = 2 open kernel's scratch 52 -> 16 bytes, s_nop
# 940 / 771 -> 846 / 801. Tile GPU tests on the variant, then three interleaved rounds on configs 4 and 5.
cd "$GRAFT_REPO_ROOT" || return 1
RG_AEAD_LIB=tools/build/librg_tmaxocc.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "tile or cfg4 or cfg5 or forged or digest or random or large" > gpurun_out/tsched_tests.log 2>&1 \
    || { echo "tests rc=$?"; tail -20 gpurun_out/tsched_tests.log; return 1; }
tail -1 gpurun_out/tsched_tests.log
bash tools/ab.sh "base tmaxocc" "cfg4 cfg5" 3
}

recipe_r5_r2l() {
# Round 5: the flattened kernel's carry power right to left with h folded in (the multiply by r^(2^i) and
# the next squaring are independent) against the commit before (tools/build_rev.sh prev): flat/forged/
# digest GPU tests, three interleaved config-3 rounds, phase stamps.
cd "$GRAFT_REPO_ROOT" || return 1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "flat or coop or forged or digest or imix or random or large" \
    > gpurun_out/r2l_tests.log 2>&1 || { echo "tests rc=$?"; tail -20 gpurun_out/r2l_tests.log; return 1; }
tail -1 gpurun_out/r2l_tests.log
bash tools/ab.sh "base prev" "cfg3" 3 || return 1
RG_AEAD_LIB=tools/build/librg_diag.so timeout -k 10 200 python tools/flat_stamps.py --workload cfg3 > gpurun_out/r5_flat_stamps_r2l.txt 2>&1 \
    || { tail -5 gpurun_out/r5_flat_stamps_r2l.txt; return 1; }
grep -v "^/opt" gpurun_out/r5_flat_stamps_r2l.txt | cut -c1-600
}

recipe_r5_restore_global() {
# Round 5: the forged-frame restore (rg_device.h restore_forged) through explicit global pointers instead of
# generic ones (the pipelined open had 16 flat_* accesses there, now none): forged/open GPU tests, then the
# bench's forged-open legs (1 % and 10 % forged) on config 2 and the tile geometry, against the commit before.
cd "$GRAFT_REPO_ROOT" || return 1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "forged or open or roundtrip" \
    > gpurun_out/rg_tests.log 2>&1 || { echo "tests rc=$?"; tail -20 gpurun_out/rg_tests.log; return 1; }
tail -1 gpurun_out/rg_tests.log
for r in 1 2; do for v in base prev; do
    if [ $v = base ]; then unset RG_AEAD_LIB; else export RG_AEAD_LIB=tools/build/librg_$v.so; fi
    timeout -k 10 200 python bench.py --workload cfg2 --steps 10 --warmup 3 --cpu-seconds 0 --no-cold > gpurun_out/rg_${v}_$r.log 2>&1 || return 1
    echo "$v $r $(grep '"value"' gpurun_out/rg_${v}_$r.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], [(f["forged_frac"], f["open_ms"], f["clean_open_ms"], f["ratio"]) for f in d["forged_open"]])')"
done; done
unset RG_AEAD_LIB
}

if [ "${1:-}" = "--list" ] || [ $# -eq 0 ]; then
    grep -A1 '^recipe_[a-z0-9_]*() {' "$SELF" | sed -n 's/^recipe_\([a-z0-9_]*\)() {/\1/p;s/^# \(.*\)/    \1/p'
    exit 0
fi
name=$1
shift
declare -F "recipe_$name" > /dev/null || { echo "no recipe $name (tools/recipes.sh --list)"; exit 2; }
"recipe_$name" "$@"
