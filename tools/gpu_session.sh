#!/bin/bash
# One GPU call that runs a list of steps in order, each under its own time limit, and stops
# at the first step that fails, times out or crashes (no GPU work after a fault).
#   bash tools/gpu_session.sh TAG step [step ...]
# steps: resident | profile | nlab | suite | bench | bench_t2 | benchsize | trace | trace_c1
set -u
TAG=$1
shift
mkdir -p gpurun_out
run() {   # name seconds command...
  local name=$1 secs=$2
  shift 2
  echo "[session] $name: $*"
  timeout -k 10 "$secs" "$@" > "gpurun_out/${TAG}_${name}.out" 2> "gpurun_out/${TAG}_${name}.err"
  local rc=$?
  echo "[session] $name rc=$rc"
  tail -3 "gpurun_out/${TAG}_${name}.out"
  if [ $rc -ne 0 ]; then
    tail -20 "gpurun_out/${TAG}_${name}.err"
    exit $rc
  fi
}
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
for step in "$@"; do
  case $step in
    resident) run resident 300 $PYT -s tests/test_gpu_ge_resident.py ;;
    profile) run profile 300 python -u tools/ge_resident_profile.py ;;
    g12) run g12 300 python -u tools/ge_resident_profile.py --modes resident --reps 3 --cells 12 ;;
    g6) run g6 300 python -u tools/ge_resident_profile.py --modes resident --reps 3 --cells 6 ;;
    q25) run q25 300 python -u tools/ge_resident_profile.py --modes resident --reps 3 --rebalance 25 ;;
    q34) run q34 300 python -u tools/ge_resident_profile.py --modes resident --reps 3 --rebalance 34 ;;
    q67) run q67 300 python -u tools/ge_resident_profile.py --modes resident --reps 3 --rebalance 67 ;;
    q80) run q80 300 python -u tools/ge_resident_profile.py --modes resident --reps 3 --rebalance 80 ;;
    x4) run x4 300 python -u tools/ge_resident_profile.py --modes resident --reps 3 --extrap 4 ;;
    x8) run x8 300 python -u tools/ge_resident_profile.py --modes resident --reps 3 --extrap 8 ;;
    x16) run x16 300 python -u tools/ge_resident_profile.py --modes resident --reps 3 --extrap 16 ;;
    ls0) run ls0 300 python -u tools/ge_resident_profile.py --modes resident,host --reps 3 --logsec 0 ;;
    g24h) run g24h 300 python -u tools/ge_resident_profile.py --modes resident,host --reps 3 ;;
    g24off) run g24off 300 python -u tools/ge_resident_profile.py --modes resident --reps 3 --rebalance 0 ;;
    stress_ls) run stress_ls 400 python -u tools/stress_logsec.py ;;
    lsl) run lsl 400 $PYT -s tests/test_gpu_ge_resident.py -k logsec_levels ;;
    g24) run g24 300 python -u tools/ge_resident_profile.py --modes resident --reps 3 ;;
    panelvar3) run panelvar3 400 env NAG=99999998 T=200 OPTS='[[1,0,0,0,200],[1,0,0,1,200]]' AIY_VARIANTS=nophilox=aiyagari_hark_amd/lib/variants/libaiyagari_nophilox.so,nolookup=aiyagari_hark_amd/lib/variants/libaiyagari_nolookup.so,noindex=aiyagari_hark_amd/lib/variants/libaiyagari_noindex.so,norecord=aiyagari_hark_amd/lib/variants/libaiyagari_norecord.so,phases=aiyagari_hark_amd/lib/variants/libaiyagari_phases.so python -u tools/panel_variants.py ;;
    panelvar1) run panelvar1 400 env NAG=1000006 T=400 OPTS='[[1,0,0,0,400],[1,0,0,1,400]]' AIY_VARIANTS=nophilox=aiyagari_hark_amd/lib/variants/libaiyagari_nophilox.so,nolookup=aiyagari_hark_amd/lib/variants/libaiyagari_nolookup.so,noindex=aiyagari_hark_amd/lib/variants/libaiyagari_noindex.so,norecord=aiyagari_hark_amd/lib/variants/libaiyagari_norecord.so,phases=aiyagari_hark_amd/lib/variants/libaiyagari_phases.so python -u tools/panel_variants.py ;;
    hphase_stress) run hphase_stress 300 env STRESS=1 AIYAGARI_LIB=aiyagari_hark_amd/lib/variants/libaiyagari_phases.so python -u tools/hist_phases.py 3 0 -1 ;;
    hphase_t2) run hphase_t2 300 env AIYAGARI_LIB=aiyagari_hark_amd/lib/variants/libaiyagari_phases.so python -u tools/hist_phases.py 24 0 -1 ;;
    trace_c4) export TMPDIR=/tmp; run trace_c4 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_trace_c4 -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --legs configs4 ;;
    trace_c3) export TMPDIR=/tmp; run trace_c3 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_trace_c3 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --legs configs3 ;;
    pull) run pull 400 $PYT -s tests/test_gpu_hist_resident.py -k "pull or rouwenhorst" ;;
    manys) run manys 400 $PYT -s tests/test_gpu_hist_resident.py -k many_states ;;
    manyge) run manyge 400 $PYT -s tests/test_gpu_parity.py -k "many_states or native_ge_search" ;;
    c4) run c4 400 python -u bench.py --legs configs4 --steps 2 --warmup 1 --no-cpu-baseline ;;
    pull7) run pull7 400 $PYT -s tests/test_gpu_hist_resident.py tests/test_gpu_ge_resident.py -k "pull" ;;
    t2pull) run t2pull 300 python -u bench.py --legs table2 --steps 10 --warmup 3 --no-cpu-baseline --hist-pull 1 ;;
    t2push) run t2push 300 python -u bench.py --legs table2 --steps 10 --warmup 3 --no-cpu-baseline --hist-pull 0 ;;
    panelfuse3) run panelfuse3 400 env NAG=99999998 T=200 OPTS='[[1,0,0,0,200],[1,0,1,0,200],[1,0,2,0,200]]' FUSE=1 python -u tools/panel_variants.py ;;
    panelnofuse3) run panelnofuse3 400 env NAG=99999998 T=200 OPTS='[[1,0,0,0,200],[1,0,1,0,200],[1,0,2,0,200]]' FUSE=0 python -u tools/panel_variants.py ;;
    t2q34) run t2q34 300 python -u bench.py --legs table2 --steps 10 --warmup 3 --no-cpu-baseline --ge-rebalance 34 ;;
    t2q67) run t2q67 300 python -u bench.py --legs table2 --steps 10 --warmup 3 --no-cpu-baseline --ge-rebalance 67 ;;
    t2q25) run t2q25 300 python -u bench.py --legs table2 --steps 10 --warmup 3 --no-cpu-baseline --ge-rebalance 25 ;;
    t2qsweep) for rep in 1 2; do for q in 55 ${QS:-45 67}; do run t2qs_${q}_$rep 300 python -u bench.py --legs table2 --steps 10 --warmup 3 --no-cpu-baseline --ge-rebalance $q; done; done ;;
    t2lh8) run t2lh8 300 python -u bench.py --legs table2 --steps 10 --warmup 3 --no-cpu-baseline --ge-loose-hist 8 ;;
    t2lh9) run t2lh9 300 python -u bench.py --legs table2 --steps 10 --warmup 3 --no-cpu-baseline --ge-loose-hist 9 ;;
    profc4) run profc4 400 python -u tools/ge_resident_profile.py --stress --reps 2 ;;
    t2lh7) run t2lh7 300 python -u bench.py --legs table2 --steps 10 --warmup 3 --no-cpu-baseline --ge-loose-hist 7 ;;
    t2lhsweep) for rep in 1 2; do for q in 8 ${LHS:-7 6}; do run t2lh_${q}_$rep 300 python -u bench.py --legs table2 --steps 10 --warmup 3 --no-cpu-baseline --ge-loose-hist $q; done; done ;;
    lgnt) for e in 1 0; do run lgnt$e 500 env ENGINE=$e NAG=99999998 T=200 OPTS='[[1,0,1,0,200]]' FUSE=0 AIY_VARIANTS=lg11=aiyagari_hark_amd/lib/variants/libaiyagari_lg11.so,lg12=aiyagari_hark_amd/lib/variants/libaiyagari_lg12.so,nt=aiyagari_hark_amd/lib/variants/libaiyagari_nt.so python -u tools/panel_variants.py; done ;;
    sortl3) run sortl3 500 env ENGINE=0 PRESORT_KEY=local NAG=99999998 T=200 OPTS='[[1,0,1,1,5],[1,0,1,1,20],[1,0,1,1,100]]' FUSE=0 python -u tools/panel_variants.py ;;
    sort3) run sort3 500 env ENGINE=0 PRESORT_KEY=la NAG=99999998 T=200 OPTS='[[1,0,1,0,20],[1,0,1,1,5],[1,0,1,1,20],[1,0,1,1,100]]' FUSE=0 python -u tools/panel_variants.py ;;
    sub8b) run sub8_16 400 python -u tools/table2_rank_subsets.py 8 16 && run sub8_24 400 python -u tools/table2_rank_subsets.py 8 24 && run sub8_48 400 python -u tools/table2_rank_subsets.py 8 48 ;;
    g3) run g3 300 python -u tools/ge_resident_profile.py --modes resident --reps 3 --cells 3 --rebalance 0 ;;
    ring3) run ring3 400 env NAG=99999998 T=200 OPTS='[[1,0,1,0,200]]' FUSE=0 AIY_VARIANTS=phases=aiyagari_hark_amd/lib/variants/libaiyagari_phases.so python -u tools/panel_variants.py ;;
    panel3) run panel3 300 env NAG=99999998 T=200 OPTS='[[1,0,1,0,200]]' FUSE=0 python -u tools/panel_variants.py ;;
    panelvar3s1) run panelvar3s1 400 env NAG=99999998 T=200 OPTS='[[1,0,1,0,200]]' FUSE=0 AIY_VARIANTS=nophilox=aiyagari_hark_amd/lib/variants/libaiyagari_nophilox.so,nolookup=aiyagari_hark_amd/lib/variants/libaiyagari_nolookup.so,phases=aiyagari_hark_amd/lib/variants/libaiyagari_phases.so python -u tools/panel_variants.py ;;
    panelshapes1) run panelshapes1 400 env NAG=1000006 T=400 OPTS='[[1,0,0,0,400],[1,0,1,0,400],[1,0,2,0,400]]' FUSE=0 python -u tools/panel_variants.py ;;
    nlab) run nlab 400 $PYT tests/test_gpu_nlab.py ;;
    fullsize) run fullsize 500 $PYT tests/test_gpu_fullsize.py ;;
    benchsize) run benchsize 500 $PYT tests/test_gpu_benchsize.py ;;
    rest) run rest 600 $PYT -m gpu tests/test_gpu_parity.py tests/test_gpu_sharded.py tests/test_gpu_stats.py ;;
    suite) run suite 1000 $PYT -m gpu tests ;;
    bench) run bench 600 python -u bench.py --steps 20 --warmup 5 ;;
    benchdef) run benchdef 900 python -u bench.py ;;
    smoke) run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    determ) run determ 300 python -u tools/hist_determinism.py ge ;;
    benchlegs) run benchlegs 600 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --legs table2,configs1,configs3,configs4 ;;
    bench_t2) run bench_t2 300 python -u bench.py --legs table2 --steps 10 --warmup 3 --no-cpu-baseline ;;
    trace) export TMPDIR=/tmp; run trace 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_trace -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --legs table2 ;;
    trace_c1) export TMPDIR=/tmp; run trace_c1 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_trace_c1 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --legs configs1 ;;
    pipet) run pipet 600 $PYT -s tests/test_gpu_ge_resident.py tests/test_gpu_benchsize.py::test_table2_bench_sweep_matches_oracle_fullsize ;;
    ab3) for v in default ${VARIANTS:-}; do lib=aiyagari_hark_amd/lib/libaiyagari.so; [ $v = default ] || lib=aiyagari_hark_amd/lib/variants/libaiyagari_$v.so; run ab3_$v 300 env AIYAGARI_LIB=$lib python -u tools/ge_resident_profile.py --modes resident --reps 3 --cells 3 --rebalance 0; done ;;
    abt2) for v in default ${VARIANTS:-}; do lib=aiyagari_hark_amd/lib/libaiyagari.so; [ $v = default ] || lib=aiyagari_hark_amd/lib/variants/libaiyagari_$v.so; run abt2_$v 300 env AIYAGARI_LIB=$lib python -u bench.py --legs table2 --steps 10 --warmup 3 --no-cpu-baseline; done ;;
    sub8) run sub8 400 python -u tools/table2_rank_subsets.py 8 32 ;;
    ph3) for v in ${PHVARIANTS:-phfusea}; do run ph3_$v 300 env AIYAGARI_LIB=aiyagari_hark_amd/lib/variants/libaiyagari_$v.so python -u tools/ge_resident_profile.py --modes resident --reps 1 --cells 3 --rebalance 0; done ;;
    sharded) run sharded 500 $PYT -s tests/test_gpu_sharded.py tests/test_gpu_benchsize.py -k "configs3 or sharded or shard or rccl" ;;
    c3pred) run c3pred 400 python -u tools/c3_shard_predict.py ;;
    abc4) for v in default ${VARIANTS:-}; do lib=aiyagari_hark_amd/lib/libaiyagari.so; [ $v = default ] || lib=aiyagari_hark_amd/lib/variants/libaiyagari_$v.so; run abc4_$v 400 env AIYAGARI_LIB=$lib python -u bench.py --legs configs4 --steps 1 --warmup 0 --no-cpu-baseline; done ;;
    dkc1) run dkc1_noisy 60 python -u tools/hist_determinism.py noisy 300 && run dkc1_nofusea 90 env AIYAGARI_LIB=aiyagari_hark_amd/lib/variants/libaiyagari_nofusea.so python -u tools/ge_resident_profile.py --modes resident --reps 1 --cells 3 --rebalance 0 && run dkc1_fusea 90 python -u tools/ge_resident_profile.py --modes resident --reps 1 --cells 3 --rebalance 0 ;;
    dpush) run dp_sweep 400 python -u tools/hist_determinism.py sweep 0 && run dp_sweep_head 400 env AIYAGARI_LIB=aiyagari_hark_amd/lib/variants/libaiyagari_headpush.so python -u tools/hist_determinism.py sweep 0 ;;
    absub8) for v in default ${VARIANTS:-}; do lib=aiyagari_hark_amd/lib/libaiyagari.so; [ $v = default ] || lib=aiyagari_hark_amd/lib/variants/libaiyagari_$v.so; run absub8_$v 300 env AIYAGARI_LIB=$lib python -u tools/table2_rank_subsets.py 8 32; done ;;
    ablegs) for v in default ${VARIANTS:-}; do lib=aiyagari_hark_amd/lib/libaiyagari.so; [ $v = default ] || lib=aiyagari_hark_amd/lib/variants/libaiyagari_$v.so; run ablegs_$v 400 env AIYAGARI_LIB=$lib python -u bench.py --legs ${LEGS:-configs1} --steps 2 --warmup 1 --no-cpu-baseline; done ;;
    c3grab) for rep in 1 2; do run c3grab_$rep 500 env NAG=99999998 T=200 OPTS='[[1,0,1,0,200]]' FUSE=0 AIY_VARIANTS=grabs=aiyagari_hark_amd/lib/variants/libaiyagari_grabs.so,head=aiyagari_hark_amd/lib/libaiyagari.so python -u tools/panel_variants.py; done ;;
    c3ab) run c3ab 500 env NAG=99999998 T=200 OPTS='[[1,0,1,0,200]]' FUSE=0 AIY_VARIANTS=c9528ed=aiyagari_hark_amd/lib/variants/libaiyagari_c9528ed.so,head=aiyagari_hark_amd/lib/libaiyagari.so${C3VARIANTS:-} python -u tools/panel_variants.py ;;
    newtests) run newtests 600 $PYT -s tests/test_gpu_ge_resident.py::test_final_ks_is_solved_at_hist_tol tests/test_gpu_parity.py::test_distribution_solve_independent_of_launch_mates tests/test_gpu_sharded.py::test_two_step_shards_equal_unsharded tests/test_gpu_benchsize.py::test_configs3_fullsize_rccl_sharded_path_matches_oracle tests/test_gpu_benchsize.py::test_configs3_fullsize_streaming_panel_matches_oracle ;;
    prof24) run prof24 300 python -u tools/ge_resident_profile.py --modes resident --reps 3 --all-evals ;;
    abt2r) for rep in 1 2; do for v in default ${VARIANTS:-}; do lib=aiyagari_hark_amd/lib/libaiyagari.so; [ $v = default ] || lib=aiyagari_hark_amd/lib/variants/libaiyagari_$v.so; run abt2_${v}_$rep 300 env AIYAGARI_LIB=$lib python -u bench.py --legs table2 --steps 10 --warmup 3 --no-cpu-baseline; done; done ;;
    t2size) run t2size 400 $PYT -s tests/test_gpu_benchsize.py::test_table2_bench_sweep_matches_oracle_fullsize ;;
    abaa) for rep in 1 2; do
            run abaa_def_$rep 300 python -u bench.py --legs table2 --steps 10 --warmup 3 --no-cpu-baseline
            for pp in ${AAP:-0}; do run abaa_p${pp}_$rep 300 python -u bench.py --legs table2 --steps 10 --warmup 3 --no-cpu-baseline --ge-anderson $pp; done
            for v in ${VARIANTS:-}; do run abaa_${v}_$rep 300 env AIYAGARI_LIB=aiyagari_hark_amd/lib/variants/libaiyagari_$v.so python -u bench.py --legs table2 --steps 10 --warmup 3 --no-cpu-baseline; done
          done ;;
    abc4aa) for rep in 1 2; do run abc4aa_def_$rep 400 python -u bench.py --legs configs4 --steps 2 --warmup 1 --no-cpu-baseline && run abc4aa_p0_$rep 400 python -u bench.py --legs configs4 --steps 2 --warmup 1 --no-cpu-baseline --ge-anderson 0; done ;;
    c4size) run c4size 600 $PYT -s tests/test_gpu_benchsize.py::test_stress_ge_matches_oracle_fullsize ;;
    abq) for rep in 1 2; do for q in ${QS:-45 65}; do run abq_q${q}_$rep 300 python -u bench.py --legs table2 --steps 10 --warmup 3 --no-cpu-baseline --ge-rebalance $q ${QEXTRA:-}; done; done ;;
    ph24) run ph24 300 env AIYAGARI_LIB=aiyagari_hark_amd/lib/variants/libaiyagari_phases.so python -u tools/ge_resident_profile.py --modes resident --reps 1 --cells 24 --rebalance 0 ;;
    c3shape) run c3shape 600 env NAG=99999998 T=200 OPTS='[[1,0,1,0,200],[1,0,3,0,200]]' FUSE=0 AIY_VARIANTS=c3pre=aiyagari_hark_amd/lib/variants/libaiyagari_c3pre.so python -u tools/panel_variants.py ;;
    c3ph) run c3ph 600 env NAG=99999998 T=200 OPTS='[[1,0,1,0,200]]' FUSE=0 AIY_VARIANTS=phases=aiyagari_hark_amd/lib/variants/libaiyagari_phases.so python -u tools/panel_variants.py ;;
    c3dg) run c3dg 600 env NAG=99999998 T=200 OPTS='[[1,0,1,0,200]]' FUSE=0 AIY_VARIANTS=dg10=aiyagari_hark_amd/lib/variants/libaiyagari_dg10.so,dg16=aiyagari_hark_amd/lib/variants/libaiyagari_dg16.so python -u tools/panel_variants.py ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "[session] done"
